"""Drop-in for the reference's train_model.py (load_dataset / train_and_evaluate) on MI355X.

``load_dataset`` (train_model.py:21-110) returns the same (X, y, class_names, feature_names) for
a frame length / shift in milliseconds and a window, but through the fused kernel: the WAVs of a
directory are decoded once per process (src/dataset.PCMDataset, kept in HBM) and every call is
one launch over all clips -- the ablation sweeps (ablation_study.py) call it once per setting.
``train_and_evaluate`` (:113-...) splits, z-scores and trains as the reference does; the KNN runs
on the device, the MLP of the reference is outside the accelerated path (src/models.py).
"""
import os
import sys

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import config  # noqa: E402
from src.dataset import PCMDataset  # noqa: E402
from src.feature_extraction import normalize_features  # noqa: E402
from src.models import create_classifier  # noqa: E402
from src.pipeline import FEATURE_NAMES  # noqa: E402

_DATASETS = {}


def dataset(data_dir):
    """The decoded, HBM-resident dataset of ``data_dir`` (decoded on first use)."""
    key = os.path.abspath(data_dir)
    if key not in _DATASETS:
        _DATASETS[key] = PCMDataset(key)
    return _DATASETS[key]


def load_dataset(data_dir, frame_length_ms=None, frame_shift_ms=None, window_type='hamming', verbose=True):
    """train_model.py:21-110 -> X [n, 15] float64, y [n], class_names, feature_names."""
    if frame_length_ms is None:
        frame_length_ms = config.FRAME_LENGTH_MS
    if frame_shift_ms is None:
        frame_shift_ms = config.FRAME_SHIFT_MS
    frame_length = int(config.SAMPLE_RATE * frame_length_ms / 1000)  # :42-43
    frame_shift = int(config.SAMPLE_RATE * frame_shift_ms / 1000)
    d = dataset(data_dir)
    X, y, ok = d.extract(frame_length, frame_shift, window_type, True, config.ENERGY_HIGH_RATIO,
                         config.ENERGY_LOW_RATIO, config.ZCR_THRESHOLD_RATIO)
    if verbose:
        print("dataset %s: %d clips (%d skipped), frame %d ms (%d samples), shift %d ms (%d samples), %s"
              % (os.path.basename(os.path.abspath(data_dir)), len(X), len(d.skipped) + int((~ok).sum()),
                 frame_length_ms, frame_length, frame_shift_ms, frame_shift, window_type))
    return X, y, list(d.class_names), list(FEATURE_NAMES)


def train_and_evaluate(X, y, classifier_type='knn', test_size=0.2, random_seed=42, verbose=True,
                       **classifier_params):
    """train_model.py:113-...: stratified split, z-score fit on train, fit, evaluate."""
    from sklearn.model_selection import train_test_split
    X_train, X_test, y_train, y_test = train_test_split(X, y, test_size=test_size, random_state=random_seed,
                                                        stratify=y)
    X_train_norm, mean, std = normalize_features(X_train)
    X_test_norm, _, _ = normalize_features(X_test, mean, std)
    if classifier_type == 'knn' and 'n_neighbors' not in classifier_params:
        classifier_params['n_neighbors'] = config.KNN_N_NEIGHBORS
    clf = create_classifier(classifier_type, **classifier_params)
    clf.fit(X_train_norm, y_train)
    res = clf.evaluate(X_test_norm, y_test)
    res['train_accuracy'] = float(np.mean(clf.predict(X_train_norm) == y_train))
    res['classifier'] = clf
    if verbose:
        print("%s: test accuracy %.4f, train accuracy %.4f" % (classifier_type, res['accuracy'],
                                                               res['train_accuracy']))
    return res
