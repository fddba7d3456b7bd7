"""GPU parity of the drop-in module surface (src/audio_processing.py, feature_extraction.py,
models.py, experiments/run_experiments.py) against the oracle."""
import os
import wave

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from conftest import golden_clip  # noqa: E402


def _write_wav(path, data, width=2, channels=1, sr=44100):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes(np.ascontiguousarray(data).tobytes())


def rel_ok(a, b, tol=1e-5):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= tol * np.abs(b) + 1e-6 * np.abs(b).mean() + 1e-30)


@pytest.mark.parametrize("vad", [True, False])
def test_process_audio_file_and_features(tmp_path, vad):
    from src.audio_processing import process_audio_file
    from src.feature_extraction import extract_features_from_frames
    from src.pipeline import create_window
    from src.synth import make_clip
    for i, (L, S, win) in enumerate([(1102, 441, "hamming"), (1024, 512, "hanning"), (1102, 441, "rectangular")]):
        x = make_clip(100 + i)
        p = tmp_path / ("c%d.wav" % i)
        _write_wav(p, x)
        frames, sr, md = process_audio_file(str(p), L, S, win, vad)
        r = oracle.process_clip(x, L, S, create_window(win, L), do_vad=vad)
        assert sr == 44100 and md["original_length"] == x.size and md["n_frames"] == r["n_frames"] == len(frames)
        if vad:
            assert (md["start_point"], md["end_point"]) == (r["start"], r["end"])
            assert md["segmented_length"] == r["end"] - r["start"]
            assert np.array_equal(md["zcr_list"], r["vad_zcr"])
            assert np.allclose(md["energy_list"], r["vad_energy"], rtol=1e-12, atol=0)
        else:
            assert "start_point" not in md
        vec, names = extract_features_from_frames(frames, "statistical")
        assert names[0] == "energy_mean" and len(names) == 15
        assert rel_ok(vec, r["feat"])
        seq, none = extract_features_from_frames(frames, "sequence")
        assert none is None and seq.shape == (r["n_frames"], 3)
        assert np.array_equal(seq[:, 2], r["seq"][:, 2]) and rel_ok(seq[:, :2], r["seq"][:, :2])
        seq2, _ = extract_features_from_frames(frames, "sequence", use_only_energy_zcr=True)
        assert seq2.shape == (r["n_frames"], 2)
        # materialised frames (device float64) reproduce the kernel's per-frame values
        fr = np.asarray(frames)
        assert fr.shape == (r["n_frames"], L)
        assert rel_ok((fr ** 2).sum(axis=1), r["seq"][:, 0])


def test_file_loop_reuses_device_buffers(tmp_path):
    """The reference's per-file loop (experiments/run_experiments.py:82-111): files of different
    lengths within one length bucket share one set of device outputs, and each result still
    equals the oracle's."""
    from src import audio_processing as AP
    from src.pipeline import create_window
    from src.synth import make_clip
    L, S = 1102, 441
    fx = AP._extractor(L, S, "hamming", True, 0.5, 0.1, 1.5)
    seen = set()
    for i, n in enumerate([41000, 43217, 44100, 42001, 44099]):  # one bucket: (40960, 49152]
        x = make_clip(300 + i)[:n]
        p = tmp_path / ("f%d.wav" % i)
        _write_wav(p, x)
        _, _, md = AP.process_audio_file(str(p), L, S)
        r = oracle.process_clip(x, L, S, create_window("hamming", L))
        assert (md["start_point"], md["end_point"], md["n_frames"]) == (r["start"], r["end"], r["n_frames"])
        seen.add(id(fx._bufs[next(iter(fx._bufs))]["feat"]))
    assert len(seen) == 1


def test_wav_formats_and_errors(tmp_path):
    from src.audio_processing import process_audio_file
    from src.pipeline import create_window
    from src.synth import make_clip
    x = make_clip(7)
    u8 = ((x.astype(np.int32) >> 8) + 128).astype(np.uint8)
    _write_wav(tmp_path / "u8.wav", u8, width=1)
    frames, _, md = process_audio_file(str(tmp_path / "u8.wav"), 1102, 441)
    r = oracle.process_clip((u8 ^ 0x80).astype(np.int16), 1102, 441, create_window("hamming", 1102))  # load_wav's uint8 wrap
    assert (md["start_point"], md["end_point"]) == (r["start"], r["end"])
    _write_wav(tmp_path / "empty.wav", np.zeros(0, np.int16))
    with pytest.raises(ValueError):
        process_audio_file(str(tmp_path / "empty.wav"), 1102, 441)
    with pytest.raises(ValueError):
        process_audio_file(str(tmp_path / "u8.wav"), 1102, 441, window_type="kaiser")


def test_array_helpers_match_numpy(golden):
    from src import audio_processing as ap
    from src.feature_extraction import compute_statistics, extract_frame_features
    x = golden_clip(golden, 3).astype(np.float64) / 32768.0
    ref_pre = x - x.mean()
    ref_pre = ref_pre / np.max(np.abs(ref_pre))
    pre = ap.preprocess(x)
    assert np.allclose(pre, ref_pre, rtol=1e-12, atol=1e-15)
    fr = ap.frame_signal(pre, 1102, 441, "hamming")
    assert fr.shape == (int(np.ceil((x.size - 1102) / 441)) + 1, 1102)
    ff = extract_frame_features(fr)
    s = np.where(fr > 0, 1.0, -1.0)
    assert np.allclose(ff["energy"], (fr ** 2).sum(axis=1), rtol=1e-12)
    assert np.array_equal(ff["zcr"], np.abs(np.diff(s, axis=1)).sum(axis=1) / 2)
    st = compute_statistics(ff["energy"])
    assert np.isclose(st["median"], np.median(ff["energy"]), rtol=1e-15)
    assert np.isclose(st["std"], np.std(ff["energy"]), rtol=1e-12)
    assert np.isclose(ap.compute_zero_crossing_rate(fr[5]), ff["zcr"][5])
    st_, en_, E, Z = ap.endpoint_detection(pre, 1102, 441)
    r = oracle.process_clip(golden_clip(golden, 3), 1102, 441, np.hamming(1102))
    assert (st_, en_) == (r["start"], r["end"])


def test_normalize_features_bitexact():
    from src.feature_extraction import normalize_features
    rng = np.random.default_rng(1)
    X = rng.normal(size=(300, 15)) * rng.uniform(0.1, 100, 15)
    X[:, 4] = 3.0  # zero std column
    Xn, m, s = normalize_features(X)
    rm, rs = X.mean(axis=0), X.std(axis=0)
    rs = np.where(rs == 0, 1, rs)
    assert np.array_equal(m, rm) and np.array_equal(s, rs) and np.array_equal(Xn, (X - rm) / rs)
    Y = rng.normal(size=(40, 15))
    Yn, m2, s2 = normalize_features(Y, m, s)
    assert np.array_equal(Yn, (Y - rm) / rs)


def test_knn_classifier_matches_sklearn_semantics(knn_golden):
    from src.models import TraditionalClassifier
    g = knn_golden
    for k in (3, 5):
        clf = TraditionalClassifier('knn', n_neighbors=k).fit(g["Xtr"], g["ytr"])
        assert np.array_equal(clf.predict(g["Xte"]), g["k%d/pred" % k])
        d, i = clf.kneighbors(g["Xte"])
        assert np.array_equal(i, g["k%d/idx" % k]) and np.array_equal(d, g["k%d/dist" % k])
        ev = clf.evaluate(g["Xte"], g["k%d/pred" % k])
        assert ev["accuracy"] == 1.0 and ev["confusion_matrix"].shape[0] == len(np.unique(g["k%d/pred" % k]))
    # arbitrary (string) labels map through sorted classes_
    lab = np.array(["cat", "dog", "emu"])[g["ytr"] % 3]
    clf = TraditionalClassifier('knn', n_neighbors=3).fit(g["Xtr"], lab)
    i0, d0, p0 = oracle.knn(g["Xtr"], (g["ytr"] % 3).astype(np.int32), g["Xte"], 3, n_classes=3)
    assert np.array_equal(clf.predict(g["Xte"]), np.array(["cat", "dog", "emu"])[p0])


def test_load_dataset_batched(tmp_path):
    from experiments.run_experiments import SpeechRecognitionExperiment
    from src.pipeline import create_window
    from src.synth import make_clip
    truth = []
    for c in range(3):
        d = tmp_path / ("class%d" % c)
        d.mkdir()
        for j in range(4):
            x = make_clip(1000 + 10 * c + j, n_samples=30000 + 997 * j, label=c, n_classes=3)
            _write_wav(d / ("s%d.wav" % j), x)
    # a file the reference skips (unsupported sample width) and one with no audio left
    with wave.open(str(tmp_path / "class1" / "bad.wav"), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(3)
        w.setframerate(44100)
        w.writeframes(b"\0" * 300)
    exp = SpeechRecognitionExperiment(str(tmp_path), str(tmp_path / "results"))
    X, y, names = exp.load_dataset("hamming", True)
    assert X.shape == (12, 15) and len(exp.skipped) == 1 and names[-1] == "zcr_median"
    from experiments.run_experiments import list_dataset
    files, _ = list_dataset(str(tmp_path))
    good = [(f, ci) for f, ci in files if not f.endswith("bad.wav")]
    from src.audio_processing import load_wav_pcm
    for row, (f, ci) in enumerate(good):
        pcm, _ = load_wav_pcm(f)
        r = oracle.process_clip(pcm, 1102, 441, create_window("hamming", 1102))
        assert y[row] == ci and rel_ok(X[row], r["feat"])
    res = exp.experiment_classifier_comparison("hamming", classifiers={"KNN": ("knn", {"n_neighbors": 3})})
    assert 0.0 <= res["KNN"]["accuracy"] <= 1.0
    assert os.path.exists(tmp_path / "results" / "exp1_classifier_comparison" / "results.json")
    # experiment_window_comparison: {window: {'KNN', 'SVM'}} (run_experiments.py:332-393)
    wres = exp.experiment_window_comparison()
    assert set(wres) == {"rectangular", "hamming", "hanning"}
    for w, r in wres.items():
        assert set(r) == {"KNN", "SVM"} and all(0.0 <= v["accuracy"] <= 1.0 for v in r.values())
    # run.py with no --experiment runs 'all' (run.py:10-135 default)
    import run
    assert run.main(["--data-dir", str(tmp_path), "--results-dir", str(tmp_path / "r2")]) == 0
    assert os.path.exists(tmp_path / "r2" / "exp2_window_comparison" / "results.json")


def test_run_py_sample_count_frames(tmp_path):
    """BASELINE configs[0]: run.py --experiment classifier at 1024 / 512 samples (not an integer-ms
    setting of config.py:35-40); every feature row against the C oracle at those frame sizes."""
    import config
    import run
    from experiments.run_experiments import list_dataset
    from src.audio_processing import load_wav_pcm
    from src.pipeline import create_window
    from src.synth import make_clip
    for c in range(3):
        d = tmp_path / ("c%d" % c)
        d.mkdir()
        for j in range(4):
            _write_wav(d / ("x%d.wav" % j), make_clip(4100 + 10 * c + j, 40000 + 997 * j, label=c, n_classes=3))
    saved = (config.FRAME_LENGTH, config.FRAME_SHIFT)
    assert run.main(["--data-dir", str(tmp_path), "--results-dir", str(tmp_path / "r"), "--experiment",
                     "classifier", "--frame-length", "1024", "--frame-shift", "512"]) == 0
    # the flags apply to that run only: config.py's values are back for the next main()
    assert (config.FRAME_LENGTH, config.FRAME_SHIFT) == saved
    exp = run.last_experiment
    files, _ = list_dataset(str(tmp_path))
    assert exp.X.shape == (len(files), 15)
    w = create_window("hamming", 1024)
    for row, (f, ci) in enumerate(files):
        r = oracle.process_clip(load_wav_pcm(f)[0], 1024, 512, w)
        assert exp.y[row] == ci and rel_ok(exp.X[row], r["feat"]), f
    assert os.path.exists(tmp_path / "r" / "exp1_classifier_comparison" / "results.json")
