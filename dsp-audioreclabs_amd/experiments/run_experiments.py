"""Experiment runner (experiments/run_experiments.py of the reference), batched on MI355X.

``load_dataset`` keeps the reference's dataset contract (class = index of the sorted
sub-directory name, files in glob order, errored files skipped: run_experiments.py:64-111) but
reads every WAV first and extracts all of them in one fused kernel launch per window type
instead of one Python loop iteration per file.  ``experiment_classifier_comparison`` /
``experiment_window_comparison`` follow :249-393 with the KNN on the device and the other
scikit-learn classifiers unchanged; plots (src/visualization.py) and the MLP are out of scope,
results are written as JSON.
"""
import json
import os
import sys
from glob import glob

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import config  # noqa: E402
from src.audio_processing import load_wav_pcm  # noqa: E402
from src.feature_extraction import normalize_features  # noqa: E402
from src.models import create_classifier  # noqa: E402
from src.pipeline import FEATURE_NAMES, FeatureExtractor  # noqa: E402


def list_dataset(data_dir):
    """[(path, class_index)] in the reference's order, and the class names."""
    classes = sorted(d for d in os.listdir(data_dir)
                     if os.path.isdir(os.path.join(data_dir, d)) and not d.startswith('.'))
    files = []
    for ci, name in enumerate(classes):
        for f in glob(os.path.join(data_dir, name, '*.wav')):
            files.append((f, ci))
    return files, classes


class SpeechRecognitionExperiment:
    def __init__(self, data_dir, results_dir):
        self.data_dir = data_dir
        self.results_dir = results_dir
        self.class_names = None
        self.X = None
        self.y = None
        self.feature_names = None
        self.skipped = []

    def load_dataset(self, window_type='hamming', do_endpoint_detection=True):
        """-> X [n, 15] float64, y [n], feature_names (run_experiments.py:45-126)."""
        files, self.class_names = list_dataset(self.data_dir)
        clips, labels, self.skipped = [], [], []
        for path, ci in files:
            try:
                pcm, _ = load_wav_pcm(path)
            except Exception as e:  # the reference skips files it cannot process (:109-111)
                self.skipped.append((path, str(e)))
                continue
            clips.append(pcm)
            labels.append(ci)
        if not clips:
            raise ValueError("no readable WAV files under %s" % self.data_dir)
        lens = np.array([c.size for c in clips], dtype=np.int64)
        off = np.zeros(len(clips) + 1, dtype=np.int64)
        off[1:] = np.cumsum(lens)
        pcm = np.concatenate(clips + [np.zeros(8, np.int16)])
        fx = FeatureExtractor(config.FRAME_LENGTH, config.FRAME_SHIFT, window_type, do_endpoint_detection,
                              config.ENERGY_HIGH_RATIO, config.ENERGY_LOW_RATIO, config.ZCR_THRESHOLD_RATIO)
        out = fx(pcm, off, max_len=int(lens.max()))
        feat = out["feat"].cpu().numpy().astype(np.float64)
        status = out["status"].cpu().numpy() & 0xFF
        keep = status == 0
        for j in np.nonzero(~keep)[0]:
            self.skipped.append((files[j][0], "status %d" % status[j]))
        self.X = feat[keep]
        self.y = np.asarray(labels)[keep]
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
        res = {}
        for w in config.WINDOW_TYPES:
            self.load_dataset(window_type=w)
            X_tr, X_te, y_tr, y_te = self.split_normalize()
            r = self.train_and_evaluate_classifier('knn', X_tr, X_te, y_tr, y_te, n_neighbors=config.KNN_N_NEIGHBORS)
            res[w] = float(r["accuracy"])
        self._save("exp2_window_comparison", res)
        return res

    def _save(self, name, obj):
        d = os.path.join(self.results_dir, name)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "results.json"), "w") as f:
            json.dump(obj, f, indent=1)
