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


def main(argv=None):
    ap = argparse.ArgumentParser(description="isolated-word recognition experiments (MI355X)")
    ap.add_argument('--data-dir', type=str, default=None)
    ap.add_argument('--results-dir', type=str, default=None)
    ap.add_argument('--experiment', type=str, default='all',
                    choices=['all', 'classifier', 'window', 'feature', 'visualize'])
    ap.add_argument('--window-type', type=str, default='hamming', choices=['rectangular', 'hamming', 'hanning'])
    args = ap.parse_args(argv)
    if args.data_dir:
        os.environ['SPEECH_DATA_DIR'] = os.path.abspath(os.path.expanduser(args.data_dir))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import config
    from experiments.run_experiments import SpeechRecognitionExperiment
    data_dir = os.environ.get('SPEECH_DATA_DIR', config.DATA_DIR)
    if not os.path.isdir(data_dir):
        print("data directory not found: %s (use --data-dir)" % data_dir)
        return 1
    exp = SpeechRecognitionExperiment(data_dir, args.results_dir or config.RESULTS_DIR)
    out = {}
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
