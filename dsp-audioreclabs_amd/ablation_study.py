#!/usr/bin/env python3
"""Drop-in for the reference's ablation_study.py (frame-length / frame-shift sweeps) on MI355X.

The reference reloads and re-processes every WAV file for each setting
(ablation_study.py:146-163, 230-247 via train_model.load_dataset).  Here the dataset is decoded
once into HBM and each setting is one fused kernel launch over all clips (train_model.py,
src/dataset.py).  Results are written as JSON (the reference's plots need matplotlib/seaborn
and are out of scope); the default classifier is the device KNN, since the reference's MLP is
outside the accelerated path.  The learning-rate sweep only concerns the MLP and is not built.

    python ablation_study.py --data-dir <dir> --experiment frame_length|frame_shift|all
"""
import argparse
import json
import os
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import config  # noqa: E402
from train_model import load_dataset, train_and_evaluate  # noqa: E402

FRAME_LENGTH_MS_RANGE = [8, 10, 12, 15, 18, 20, 25, 30, 35, 40, 45, 50]  # config.py:81
FRAME_SHIFT_MS_RANGE = [3, 5, 7, 8, 10, 12, 15, 18, 20, 25, 30]  # config.py:85


def _sweep(data_dir, name, values, kw_of, classifier_type, save_dir, verbose):
    results = {}
    for v in values:
        X, y, class_names, _ = load_dataset(data_dir, window_type='hamming', verbose=verbose, **kw_of(v))
        r = train_and_evaluate(X, y, classifier_type=classifier_type, verbose=verbose)
        results[v] = {'accuracy': float(r['accuracy']), 'train_accuracy': float(r['train_accuracy']),
                      'confusion_matrix': r['confusion_matrix'].tolist()}
    if save_dir:
        os.makedirs(save_dir, exist_ok=True)
        with open(os.path.join(save_dir, 'results.json'), 'w') as f:
            json.dump({'experiment': name, 'dataset': os.path.basename(os.path.abspath(data_dir)),
                       'classifier': classifier_type, 'results': {str(k): v for k, v in results.items()}},
                      f, indent=1)
    return results


def ablation_frame_length(data_dir=None, frame_lengths_ms=None, classifier_type='knn', save_dir=None,
                          verbose=True):
    """ablation_study.py:112-193: accuracy per frame length (ms), frame shift from config."""
    data_dir = data_dir or config.DATA_DIR
    save_dir = save_dir if save_dir is not None else os.path.join(config.RESULTS_DIR, 'ablation_frame_length')
    return _sweep(data_dir, 'frame_length_ms', frame_lengths_ms or FRAME_LENGTH_MS_RANGE,
                  lambda v: {'frame_length_ms': v}, classifier_type, save_dir, verbose)


def ablation_frame_shift(data_dir=None, frame_shifts_ms=None, classifier_type='knn', save_dir=None,
                         verbose=True):
    """ablation_study.py:196-277: accuracy per frame shift (ms), frame length from config."""
    data_dir = data_dir or config.DATA_DIR
    save_dir = save_dir if save_dir is not None else os.path.join(config.RESULTS_DIR, 'ablation_frame_shift')
    return _sweep(data_dir, 'frame_shift_ms', frame_shifts_ms or FRAME_SHIFT_MS_RANGE,
                  lambda v: {'frame_shift_ms': v}, classifier_type, save_dir, verbose)


def main(argv=None):
    ap = argparse.ArgumentParser(description="frame length / shift ablations (MI355X)")
    ap.add_argument('--data-dir', type=str, default=None)
    ap.add_argument('--experiment', default='all', choices=['all', 'frame_length', 'frame_shift'])
    ap.add_argument('--classifier', default='knn', choices=['knn', 'svm', 'naive_bayes', 'decision_tree'])
    ap.add_argument('--results-dir', type=str, default=None)
    a = ap.parse_args(argv)
    data_dir = os.path.abspath(os.path.expanduser(a.data_dir)) if a.data_dir else config.DATA_DIR
    if not os.path.isdir(data_dir):
        print("data directory not found: %s (use --data-dir)" % data_dir)
        return 1
    rd = a.results_dir or config.RESULTS_DIR
    out = {}
    if a.experiment in ('all', 'frame_length'):
        out['frame_length'] = ablation_frame_length(data_dir, classifier_type=a.classifier,
                                                    save_dir=os.path.join(rd, 'ablation_frame_length'))
    if a.experiment in ('all', 'frame_shift'):
        out['frame_shift'] = ablation_frame_shift(data_dir, classifier_type=a.classifier,
                                                  save_dir=os.path.join(rd, 'ablation_frame_shift'))
    print({k: {kk: vv['accuracy'] for kk, vv in v.items()} for k, v in out.items()})
    return 0


if __name__ == '__main__':
    sys.exit(main())
