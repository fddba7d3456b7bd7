#!/usr/bin/env python3
"""Command line of the reference's run.py (run.py:10-135) on MI355X.

    python run.py --data-dir <dir with one sub-directory of WAVs per class> [--experiment all]

'all' (the reference's default) runs the classifier and window comparisons; the reference's
'feature' and 'visualize' experiments only draw plots (src/visualization.py, out of scope) and are
accepted and reported as such.
"""
import argparse
import os
import sys

last_experiment = None


def main(argv=None):
    ap = argparse.ArgumentParser(description="isolated-word recognition experiments (MI355X)")
    ap.add_argument('--data-dir', type=str, default=None)
    ap.add_argument('--results-dir', type=str, default=None)
    ap.add_argument('--experiment', type=str, default='all',
                    choices=['all', 'classifier', 'window', 'feature', 'visualize'])
    ap.add_argument('--window-type', type=str, default='hamming', choices=['rectangular', 'hamming', 'hanning'])
    # frame sizes in samples (config.FRAME_LENGTH / FRAME_SHIFT; BASELINE configs[0]: 1024 / 512)
    ap.add_argument('--frame-length', type=int, default=None, help='frame length in samples')
    ap.add_argument('--frame-shift', type=int, default=None, help='frame shift in samples')
    args = ap.parse_args(argv)
    if args.data_dir:
        os.environ['SPEECH_DATA_DIR'] = os.path.abspath(os.path.expanduser(args.data_dir))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import config
    from experiments.run_experiments import SpeechRecognitionExperiment
    global last_experiment
    for name, v in (('--frame-length', args.frame_length), ('--frame-shift', args.frame_shift)):
        if v is not None and v < 1:
            ap.error('%s must be positive' % name)
    # the frame sizes apply to this run only: config's module values are restored on return, so a
    # later main() in the same process without the flags gets config.py's defaults again
    saved = (config.FRAME_LENGTH, config.FRAME_SHIFT)
    try:
        if args.frame_length is not None:
            config.FRAME_LENGTH = args.frame_length
        if args.frame_shift is not None:
            config.FRAME_SHIFT = args.frame_shift
        return _run(args, config, SpeechRecognitionExperiment)
    finally:
        config.FRAME_LENGTH, config.FRAME_SHIFT = saved


def _run(args, config, SpeechRecognitionExperiment):
    global last_experiment
    data_dir = os.environ.get('SPEECH_DATA_DIR', config.DATA_DIR)
    if not os.path.isdir(data_dir):
        print("data directory not found: %s (use --data-dir)" % data_dir)
        return 1
    exp = SpeechRecognitionExperiment(data_dir, args.results_dir or config.RESULTS_DIR)
    last_experiment = exp  # the last run's data (X, y), for callers that drive main() in process
    out = {'frame_length': config.FRAME_LENGTH, 'frame_shift': config.FRAME_SHIFT}
    if args.experiment in ('all', 'classifier'):
        res = exp.experiment_classifier_comparison(window_type=args.window_type)
        out['classifier'] = {k: float(v['accuracy']) for k, v in res.items()}
    if args.experiment in ('all', 'window'):
        res = exp.experiment_window_comparison()
        out['window'] = {w: {c: float(r['accuracy']) for c, r in rw.items()} for w, rw in res.items()}
    if args.experiment in ('feature', 'visualize'):
        print("experiment '%s' draws plots only (src/visualization.py): not part of the accelerated path"
              % args.experiment)
    print(out)
    return 0

if __name__ == '__main__':
    sys.exit(main())
