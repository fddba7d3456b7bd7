#!/usr/bin/env python3
"""Drop-in for the reference's compare_feature_methods.py (statistical 15-d vs padded E+ZCR
sequence features, then the same classifiers on both).

The reference walks the dataset twice, one file at a time, once per method (:43-64, :79-104),
and pads each sequence on the host (:106-115).  Here the dataset is decoded once into HBM
(src/dataset.PCMDataset) and ONE fused launch returns both the statistical matrix and the
per-frame sequences, already zero-padded to the longest sequence (PCMDataset.extract_both).
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


# the reference's classifier table (compare_feature_methods.py:147-151)
CLASSIFIERS = {
    'KNN': ('knn', {'n_neighbors': 3}),
    'SVM': ('svm', {'C': 1.0, 'kernel': 'rbf'}),
    'Decision Tree': ('decision_tree', {}),
}


def load_both_methods(data_dir=None, frame_length=None, frame_shift=None, window_type='hamming'):
    """:27-122 -> (X_statistical [n, 15], X_sequences_padded [n, max_len, 2], y, lengths)."""
    ds = PCMDataset(data_dir or config.DATA_DIR)
    X_stat, y, X_seq, lengths = ds.extract_both(frame_length or config.FRAME_LENGTH,
                                                frame_shift or config.FRAME_SHIFT, window_type,
                                                do_endpoint_detection=True, use_only_energy_zcr=True)
    return X_stat, X_seq, y, lengths


def compare(data_dir=None, classifiers=None, test_size=0.2, random_state=42):
    """:124-214: each classifier on both feature sets, the reference's split and normalisation
    -> {classifier: {'statistical': acc, 'sequence': acc, 'diff': sequence - statistical}}.
    KNN on the flattened sequences (2 x max_frames columns) runs on the device like the 15-d
    case (dsp_knn_classify's chunked high-dimensional screen + fp64 re-rank)."""
    from sklearn.model_selection import train_test_split
    X_stat, X_seq, y, _ = load_both_methods(data_dir)
    X_flat = X_seq.reshape(len(X_seq), -1)
    Xs_tr, Xs_te, y_tr, y_te = train_test_split(X_stat, y, test_size=test_size, random_state=random_state,
                                                stratify=y)
    Xq_tr, Xq_te, _, _ = train_test_split(X_flat, y, test_size=test_size, random_state=random_state, stratify=y)
    Xs_tr, m, sd = normalize_features(Xs_tr)
    Xs_te, _, _ = normalize_features(Xs_te, m, sd)
    Xq_tr, m, sd = normalize_features(Xq_tr)
    Xq_te, _, _ = normalize_features(Xq_te, m, sd)
    results = {}
    for name, (kind, params) in (classifiers or CLASSIFIERS).items():
        acc = {}
        for method, (tr, te) in (("statistical", (Xs_tr, Xs_te)), ("sequence", (Xq_tr, Xq_te))):
            clf = create_classifier(kind, **params)
            clf.fit(tr, y_tr)
            acc[method] = float(clf.evaluate(te, y_te)['accuracy'])
        results[name] = {'statistical': acc['statistical'], 'sequence': acc['sequence'],
                         'diff': acc['sequence'] - acc['statistical']}
    return results


if __name__ == "__main__":
    res = compare()
    for name, r in res.items():
        print("%-15s statistical %.4f  sequence %.4f  diff %+.4f" % (name, r['statistical'], r['sequence'], r['diff']))
    print("mean  statistical %.4f  sequence %.4f" % (np.mean([r['statistical'] for r in res.values()]),
                                                      np.mean([r['sequence'] for r in res.values()])))
