"""Experiment runner (experiments/run_experiments.py of the reference), batched on MI355X.

``load_dataset`` keeps the reference's dataset contract (class = index of the sorted
sub-directory name, files in glob order, errored files skipped: run_experiments.py:64-111) but
decodes every WAV once (src/dataset.PCMDataset: host threads, one pinned upload) and extracts all
of them in one fused kernel launch per window type instead of one Python loop iteration per
file; the window comparison reuses the HBM-resident PCM.  ``experiment_classifier_comparison`` /
``experiment_window_comparison`` follow :249-393 with the KNN on the device and the other
scikit-learn classifiers unchanged; plots (src/visualization.py) and the MLP are out of scope,
results are written as JSON.
"""
import json
import os
import sys

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import config  # noqa: E402
from src.dataset import PCMDataset, list_dataset  # noqa: E402,F401
from src.feature_extraction import normalize_features  # noqa: E402
from src.models import create_classifier  # noqa: E402
from src.pipeline import FEATURE_NAMES  # noqa: E402


class SpeechRecognitionExperiment:
    def __init__(self, data_dir, results_dir):
        self.data_dir = data_dir
        self.results_dir = results_dir
        self.class_names = None
        self.X = None
        self.y = None
        self.feature_names = None
        self.skipped = []
        self._data = None  # PCMDataset, decoded once per runner

    def load_dataset(self, window_type='hamming', do_endpoint_detection=True):
        """-> X [n, 15] float64, y [n], feature_names (run_experiments.py:45-126)."""
        if self._data is None:
            self._data = PCMDataset(self.data_dir)
            self.class_names = self._data.class_names
        d = self._data
        X, y, ok = d.extract(config.FRAME_LENGTH, config.FRAME_SHIFT, window_type, do_endpoint_detection,
                             config.ENERGY_HIGH_RATIO, config.ENERGY_LOW_RATIO, config.ZCR_THRESHOLD_RATIO)
        self.skipped = list(d.skipped) + [(d.files[j][0], "processing failed") for j in np.nonzero(~ok)[0]]
        self.X, self.y = X, y
        self.feature_names = list(FEATURE_NAMES)
        return self.X, self.y, self.feature_names

    def split_normalize(self):
        from sklearn.model_selection import train_test_split
        X_tr, X_te, y_tr, y_te = train_test_split(self.X, self.y, test_size=config.TEST_SIZE,
                                                  random_state=config.RANDOM_SEED, stratify=self.y)
        X_tr, mean, std = normalize_features(X_tr)
        X_te, _, _ = normalize_features(X_te, mean, std)
        return X_tr, X_te, y_tr, y_te

    def train_and_evaluate_classifier(self, classifier_type, X_train, X_test, y_train, y_test, **kwargs):
        clf = create_classifier(classifier_type, **kwargs)
        clf.fit(X_train, y_train)
        return clf.evaluate(X_test, y_test)

    def experiment_classifier_comparison(self, window_type='hamming', classifiers=None):
        if self.X is None:
            self.load_dataset(window_type=window_type)
        X_tr, X_te, y_tr, y_te = self.split_normalize()
        classifiers = classifiers or {
            'KNN': ('knn', {'n_neighbors': config.KNN_N_NEIGHBORS}),
            'Naive Bayes': ('naive_bayes', {}),
            'Decision Tree': ('decision_tree', {}),
            'SVM': ('svm', {'C': config.SVM_C, 'kernel': config.SVM_KERNEL}),
        }
        res = {name: self.train_and_evaluate_classifier(t, X_tr, X_te, y_tr, y_te, **kw)
               for name, (t, kw) in classifiers.items()}
        self._save("exp1_classifier_comparison", {k: {"accuracy": float(v["accuracy"])} for k, v in res.items()})
        return res

    def experiment_window_comparison(self):
        """:332-393 -> {window_type: {classifier: evaluate() results}} for KNN and SVM (the
        reference's MLP entry is the out-of-scope torch MLP).  Every window re-runs load_dataset,
        i.e. one fused launch over the HBM-resident PCM."""
        window_results = {}
        classifiers = {'KNN': ('knn', {'n_neighbors': config.KNN_N_NEIGHBORS}),
                       'SVM': ('svm', {'C': config.SVM_C})}
        for w in config.WINDOW_TYPES:
            self.load_dataset(window_type=w)
            X_tr, X_te, y_tr, y_te = self.split_normalize()
            window_results[w] = {name: self.train_and_evaluate_classifier(kind, X_tr, X_te, y_tr, y_te, **params)
                                 for name, (kind, params) in classifiers.items()}
        self._save("exp2_window_comparison",
                   {w: {c: float(r['accuracy']) for c, r in res.items()} for w, res in window_results.items()})
        return window_results

    def _save(self, name, obj):
        d = os.path.join(self.results_dir, name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "results.json"), "w") as f:
            json.dump(obj, f, indent=1)
