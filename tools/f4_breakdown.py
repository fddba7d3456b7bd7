#!/usr/bin/env python3
"""Row f4 decided by measurement: end-to-end time of
``run.py --experiment classifier`` on a synthetic isolated-word dataset (--files WAVs, 10 classes,
written as 16-bit mono 44.1 kHz files into a temporary directory), with a per-stage breakdown of the
same code path (experiments/run_experiments.py): decode + upload, fused extraction, stratified
split (scikit-learn train_test_split, /root/reference/experiments/run_experiments.py:265-270),
z-score (device), KNN (device), Naive Bayes / Decision Tree / SVM (scikit-learn), result files.
Prints one JSON line.  Needs the GPU (the extraction and KNN run there).

    python tools/f4_breakdown.py [--files 2000]
"""
import argparse
import json
import os
import sys
import tempfile
import time
import wave

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dsp-audioreclabs_amd")
sys.path.insert(0, PKG)


def write_dataset(root, n_files, n_classes=10):
    from src.synth import make_clip
    rng = np.random.default_rng(0)
    for c in range(n_classes):
        os.makedirs(os.path.join(root, "class_%02d" % c), exist_ok=True)
    for i in range(n_files):
        c = i % n_classes
        n = int(rng.integers(30000, 60000))  # 0.7-1.4 s
        pcm = make_clip(10000 + i, n, label=c, n_classes=n_classes)
        with wave.open(os.path.join(root, "class_%02d" % c, "u%05d.wav" % i), "wb") as w:
            w.setnchannels(1)
            w.setsampwidth(2)
            w.setframerate(44100)
            w.writeframes(pcm.tobytes())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=2000)
    args = ap.parse_args()
    import torch
    tmp = tempfile.mkdtemp(prefix="f4_")
    data, res = os.path.join(tmp, "data"), os.path.join(tmp, "results")
    write_dataset(data, args.files)
    os.environ["SPEECH_DATA_DIR"] = data
    import config
    import run
    from experiments.run_experiments import SpeechRecognitionExperiment

    # warm the device path once on a few files (kernel load, allocator) so the stages time steady state
    sub = os.path.join(tmp, "warm")
    os.makedirs(os.path.join(sub, "a"))
    os.makedirs(os.path.join(sub, "b"))
    for k, dst in enumerate(("a", "b", "a", "b", "a", "b")):
        os.link(os.path.join(data, "class_%02d" % (k % 10), "u%05d.wav" % k), os.path.join(sub, dst, "w%d.wav" % k))
    SpeechRecognitionExperiment(sub, os.path.join(tmp, "wres")).load_dataset()

    # end to end, as a user runs it
    t0 = time.perf_counter()
    rc = run.main(["--data-dir", data, "--results-dir", res, "--experiment", "classifier"])
    total = time.perf_counter() - t0
    assert rc == 0

    # the same path stage by stage
    st = {}
    sync = torch.cuda.synchronize

    def tick(name, fn):
        sync()
        t = time.perf_counter()
        out = fn()
        sync()
        st[name] = time.perf_counter() - t
        return out

    exp = SpeechRecognitionExperiment(data, res)
    from src.dataset import PCMDataset
    exp._data = tick("decode_upload", lambda: PCMDataset(data))
    exp.class_names = exp._data.class_names
    tick("extraction", lambda: exp.load_dataset("hamming"))
    from sklearn.model_selection import train_test_split
    from src.feature_extraction import normalize_features
    X_tr, X_te, y_tr, y_te = tick("split", lambda: train_test_split(exp.X, exp.y, test_size=config.TEST_SIZE,
                                                                   random_state=config.RANDOM_SEED, stratify=exp.y))

    def zs():
        a, m, s = normalize_features(X_tr)
        b, _, _ = normalize_features(X_te, m, s)
        return a, b
    X_tr, X_te = tick("zscore", zs)
    for name, kind, kw in (("knn", "knn", {"n_neighbors": config.KNN_N_NEIGHBORS}), ("naive_bayes", "naive_bayes", {}),
                           ("decision_tree", "decision_tree", {}),
                           ("svm", "svm", {"C": config.SVM_C, "kernel": config.SVM_KERNEL})):
        tick(name, lambda: exp.train_and_evaluate_classifier(kind, X_tr, X_te, y_tr, y_te, **kw))
    tick("save_results", lambda: exp._save("exp1_classifier_comparison", {"k": 1}))
    staged = sum(st.values())
    print(json.dumps({"what": "run.py --experiment classifier, %d synthetic WAVs (10 classes, 0.7-1.4 s)" % args.files,
                      "end_to_end_s": round(total, 4), "stages_s": {k: round(v, 5) for k, v in st.items()},
                      "stages_sum_s": round(staged, 4),
                      "share": {k: round(v / staged, 4) for k, v in st.items()}}), flush=True)


if __name__ == "__main__":
    main()
