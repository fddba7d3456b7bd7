"""Pin the C oracle to the reference: bit-exact against golden vectors produced by
importing the reference's own src/ (tests/golden/make_golden.py)."""
import numpy as np
import pytest

import oracle
from conftest import golden_clip, golden_keys


def test_np_sum_matches_numpy():
    rng = np.random.default_rng(0)
    for n in list(range(0, 300)) + [1024, 1102, 8191, 8192, 8193, 20000, 44100]:
        a = rng.standard_normal(n) * np.exp(rng.standard_normal(n) * 3)
        assert oracle.np_sum(a) == np.sum(a), n


def test_statistics_match_numpy():
    rng = np.random.default_rng(1)
    for n in [1, 2, 3, 7, 8, 9, 64, 99, 100, 1000]:
        a = rng.standard_normal(n) * 10
        want = [np.mean(a), np.std(a), np.max(a), np.min(a), np.median(a)]
        assert np.array_equal(oracle.compute_statistics(a), want), n


def test_pipeline_bit_exact_vs_reference(golden):
    names = golden["clip_names"]
    for key, L, S, wname, vad in golden_keys(golden):
        window = golden["window/%s_%d" % (wname, L)]
        assert np.array_equal(window, {"rectangular": np.ones, "hamming": np.hamming,
                                       "hanning": np.hanning}[wname](L))
        feats = golden[key + "/feat"]
        fo = golden[key + "/frame_off"]
        for i in range(len(names)):
            r = oracle.process_clip(golden_clip(golden, i), L, S, window, do_vad=bool(vad))
            assert r["status"] == golden[key + "/status"][i]
            if r["status"]:
                continue
            ctx = (key, names[i])
            assert np.array_equal(r["feat"], feats[i]), ctx
            assert r["n_frames"] == golden[key + "/n_frames"][i], ctx
            seq = r["seq"]
            assert np.array_equal(seq[:, 0], golden[key + "/frame_energy"][fo[i]:fo[i + 1]]), ctx
            assert np.array_equal(seq[:, 1], golden[key + "/frame_magnitude"][fo[i]:fo[i + 1]]), ctx
            assert np.array_equal(seq[:, 2], golden[key + "/frame_zcr"][fo[i]:fo[i + 1]]), ctx
            if vad:
                vo = golden[key + "/vad_off"]
                assert (r["start"], r["end"]) == tuple(golden[key + "/start_end"][i]), ctx
                assert np.array_equal(r["vad_energy"], golden[key + "/vad_energy"][vo[i]:vo[i + 1]]), ctx
                assert np.array_equal(r["vad_zcr"], golden[key + "/vad_zcr"][vo[i]:vo[i + 1]]), ctx


def test_float64_stereo_path(golden):
    from src.audio_processing import decode_pcm_bytes
    raw = golden["wav/u8_stereo/raw"]
    x, _, _ = decode_pcm_bytes(raw.tobytes(), 1, 2)
    assert np.array_equal(x, golden["wav/u8_stereo/decoded"])
    win = np.hamming(1102)
    r = oracle.process_clip(x, 1102, 441, win)
    assert np.array_equal(r["feat"], golden["wav/u8_stereo/feat"])
    assert (r["start"], r["end"]) == tuple(golden["wav/u8_stereo/start_end"])
    raw = golden["wav/s16_stereo_clip/raw"]
    x, _, _ = decode_pcm_bytes(raw.tobytes(), 2, 2)
    r = oracle.process_clip(x, 1102, 441, win)
    assert np.array_equal(r["feat"], golden["wav/s16_stereo_clip/feat"])
    assert (r["start"], r["end"]) == tuple(golden["wav/s16_stereo_clip/start_end"])


def test_zscore_matches_reference(knn_golden):
    g = knn_golden
    mu, sd = oracle.zscore_fit(g["X"])
    assert np.array_equal(mu, g["mu"]) and np.array_equal(np.where(sd == 0, 1, sd), g["sd"])


@pytest.mark.parametrize("k", [3, 5])
def test_knn_oracle_matches_sklearn(knn_golden, k):
    g = knn_golden
    idx, dist, pred = oracle.knn(g["Xtr"], g["ytr"], g["Xte"], k, n_classes=10)
    assert np.array_equal(idx, g["k%d/idx" % k])
    assert np.array_equal(dist, g["k%d/dist" % k])
    assert np.array_equal(pred, g["k%d/pred" % k])


def test_knn_oracle_self_query(knn_golden):
    g = knn_golden
    X = g["Xtr"][:800]
    idx, dist, _ = oracle.knn(X, g["ytr"][:800], X, 5, n_classes=10, self_offset=0)
    assert np.array_equal(idx, g["self5/idx"])
    assert np.array_equal(dist, g["self5/dist"])


def test_np_reference_bit_exact(golden):
    """oracle/np_reference.py (the reference's per-clip numpy loop, bench.py's
    cpu_baseline_reference_semantics leg) reproduces the reference's golden outputs bit for bit."""
    import np_reference
    names = golden["clip_names"]
    for key, L, S, wname, vad in golden_keys(golden):
        window = golden["window/%s_%d" % (wname, L)]
        for i in range(len(names)):
            st, feat, s0, s1, nf = np_reference.process_clip(golden_clip(golden, i), L, S, window, do_vad=bool(vad))
            assert st == golden[key + "/status"][i], (key, names[i])
            if st:
                continue
            assert np.array_equal(feat, golden[key + "/feat"][i]), (key, names[i])
            assert nf == golden[key + "/n_frames"][i], (key, names[i])
            if vad:
                assert (s0, s1) == tuple(golden[key + "/start_end"][i]), (key, names[i])
