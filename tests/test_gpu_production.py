"""GPU parity at production batch sizes: the persistent multi-clip loop the benchmark times.

The extraction grid is persistent (three workgroups per CU, 768 on MI355X): workgroup w takes its
first chunk of clips by its own index, then claims chunks from a launch-wide queue; these tests
launch far more clips than workgroups, so every workgroup processes many clips in sequence (LDS
summaries and output staging reused, several near ties deferred to the exact kernel), and compare
everything with the C oracle (reference algorithm:
src/audio_processing.py:336-396, src/feature_extraction.py:12-88).  They also simulate the
8-rank sharding of BASELINE configs[3]/[4] on one GPU: shards processed
separately and concatenated must equal the single launch.

Tolerances as in test_gpu_extract.py (north star): endpoints, frame counts, status bit-exact;
15-d features within 1e-5 relative (+1e-6 of the sequence's magnitude for std/min of
near-constant sequences).
"""
import numpy as np
import pytest

import oracle
from test_gpu_extract import feat_close

pytestmark = pytest.mark.gpu

L, S = 1102, 441


def grid():
    """The fused kernel's persistent grid: EXTRACT_WG_PER_CU (3) workgroups per CU."""
    import torch
    return 3 * torch.cuda.get_device_properties(0).multi_processor_count


def near_tie_clip(n=44100, A=3000):
    """A clip whose first VAD frame energy equals T1 = p90 / 2 exactly at (1102, 441): a +-A
    square wave (every full frame: energy L in normalised units, so p90 = L) opened by the
    period-4 pattern (0, A, -A, 0), in which frame 0 holds exactly 551 = L / 2 nonzero samples
    while frame 1 holds 552.  Mean 0 and peak A exactly, so the energies are exact: the certified
    scan must flag frame 0 and redo the clip in numpy's exact order."""
    x = np.empty(n, np.int64)
    x[0::2], x[1::2] = A, -A
    x[:4000] = np.tile(np.array([0, A, -A, 0]), 1000)
    return x.astype(np.int16)


def _check(out, clips, w, vad=True, idx=None):
    idx = range(len(clips)) if idx is None else idx
    sel = list(idx)
    off = np.zeros(len(sel) + 1, np.int64)
    off[1:] = np.cumsum([clips[i].size for i in sel])
    flat = np.concatenate([clips[i] for i in sel] + [np.zeros(8, np.int16)])
    ref = oracle.process_batch(flat, off, L, S, w, do_vad=vad, nthreads=16)
    st = out["status"][sel] & 0xFF
    assert np.array_equal(st, ref["status"]), np.nonzero(st != ref["status"])[0][:10]
    ok = ref["status"] == 0
    se, nf = out["start_end"][sel], out["n_frames"][sel]
    bad = np.nonzero((se != ref["start_end"]).any(1) & ok)[0]
    assert bad.size == 0, ("start_end", [sel[i] for i in bad[:10]])
    bad = np.nonzero((nf != ref["n_frames"]) & ok)[0]
    assert bad.size == 0, ("n_frames", [sel[i] for i in bad[:10]])
    fb = feat_close(out["feat"][sel][ok], ref["feat"][ok])
    assert not fb.any(), ("feat", np.nonzero(fb.any(1))[0][:10])
    return ref


def test_production_batch_2000_ragged_and_near_ties():
    """2000 clips of BASELINE configs[1] (Hamming, 1102/441, VAD) with empty, short, ragged and
    near-tie clips scattered; four near-tie clips G / 2 apart in the first chunks of four different
    workgroups (round 1's static split put such clips in one workgroup's redo list)."""
    import torch
    from src.pipeline import FeatureExtractor, create_window
    from src.synth import make_batch
    B = 2000
    G = grid()
    ties = [3 + j * (G // 2) for j in range(4)]
    assert ties[-1] < B
    base = make_batch(B, base_seed=500)
    clips = [base[i] for i in range(B)]
    rng = np.random.default_rng(5)
    for i in rng.choice(B, 60, replace=False):  # ragged / short / degenerate lengths
        n = int(rng.choice([0, 1, 7, 500, 1101, 1102, 1103, 2000, 9000, 30001, 44099]))
        clips[i] = clips[i][:n].copy()
    for i in ties:
        clips[i] = near_tie_clip()
    clips[17] = np.zeros(44100, np.int16)  # silence: no high-energy frame
    off = np.zeros(B + 1, np.int64)
    off[1:] = np.cumsum([c.size for c in clips])
    pcm = np.concatenate(clips + [np.zeros(8, np.int16)])
    fx = FeatureExtractor(L, S, "hamming", True)
    out = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm).cuda(), off).items()}
    _check(out, clips, create_window("hamming", L))
    redo = (out["status"] >> 8) & 1
    assert redo[ties].all(), "near ties were not redone exactly"


@pytest.mark.parametrize("win", ["hamming", "hanning", "rectangular"])
def test_production_12500_per_rank_batch(win):
    """The per-rank batch of configs[3] (12 500 x 1 s), generated on the device; every status
    checked and a strided subset of 1 042 clips compared with the oracle."""
    import torch
    from src.pipeline import FeatureExtractor, create_window
    from src.synth import make_batch_device
    B = 12500
    x = make_batch_device(B, "cuda", base_seed=77)
    fx = FeatureExtractor(L, S, win, True)
    out = {k: v.cpu().numpy() for k, v in fx(x).items()}
    assert not (out["status"] & 0xFF).any()
    host = x.cpu().numpy()
    clips = [host[i] for i in range(B)]
    _check(out, clips, create_window(win, L), idx=range(0, B, 12))


def test_large_batch_one_launch():
    """More clips than the persistent grid's slots x 256 in one launch (round 3 chunked launches at
    that boundary; the clip queue's chunk counters now run far past it): clips on both sides of it
    and at the end match the oracle."""
    import torch
    from src.pipeline import FeatureExtractor, create_window
    from src.synth import make_batch_device
    G = grid()
    cap = G * 256
    B, n = cap + 9000, 1800
    x = make_batch_device(B, "cuda", base_seed=3, n_samples=n)
    fx = FeatureExtractor(L, S, "hamming", True)
    out = {k: v.cpu().numpy() for k, v in fx(x).items()}
    assert not (out["status"] & 0xFF).any()
    host = x.cpu().numpy()
    idx = sorted(set(range(0, B, 257)) | set(range(cap - 40, cap + 40)) | set(range(B - 40, B)))
    _check(out, [host[i] for i in range(B)], create_window("hamming", L), idx=idx)


def test_sharded_extraction_equals_single_launch():
    """configs[3] on one GPU: 8 simulated ranks, each extracting its shard_range block; the
    concatenation equals the single launch bit for bit."""
    import torch
    from src.distributed import shard_range
    from src.pipeline import FeatureExtractor
    from src.synth import make_batch_device
    B, P = 6000, 8
    x = make_batch_device(B, "cuda", base_seed=9)
    fx = FeatureExtractor(L, S, "hamming", True)
    full = {k: v.clone() for k, v in fx(x).items()}
    parts = []
    for r in range(P):
        lo, hi = shard_range(B, r, P)
        parts.append({k: v.clone() for k, v in fx(x[lo:hi]).items()})
    for k in full:
        cat = torch.cat([p_[k] for p_ in parts])
        assert torch.equal(cat, full[k]), k


def test_sharded_knn_self_query_equals_single():
    """configs[4] on one GPU: query shards with self_offset = lo (what every rank but 0 runs in
    knn_sharded), concatenated, equal the full self-query and the oracle."""
    import torch
    from src.distributed import shard_range
    from src.pipeline import knn_classify
    rng = np.random.default_rng(4)
    n, d, P, k = 20000, 15, 8, 5
    centres = rng.standard_normal((10, d)) * 1.5
    y = rng.integers(0, 10, n).astype(np.int32)
    X = centres[y] + rng.standard_normal((n, d))
    X = (X - X.mean(0)) / X.std(0)
    Xd, yd = torch.as_tensor(X, device="cuda"), torch.as_tensor(y, device="cuda")
    i_full, d_full, p_full = knn_classify(Xd, yd, Xd, k, self_offset=0)
    idx, dist, pred = [], [], []
    for r in range(P):
        lo, hi = shard_range(n, r, P)
        i_, d_, p_ = knn_classify(Xd, yd, Xd[lo:hi], k, self_offset=lo)
        idx.append(i_)
        dist.append(d_)
        pred.append(p_)
    assert torch.equal(torch.cat(idx), i_full)
    assert torch.equal(torch.cat(dist), d_full)
    assert torch.equal(torch.cat(pred), p_full)
    lo, hi = shard_range(n, 3, P)  # one rank's shard against the oracle (self excluded)
    i0, d0, p0 = oracle.knn(X, y, X[lo:hi], k, n_classes=10, self_offset=lo)
    assert np.array_equal(i_full.cpu().numpy()[lo:hi], i0)
    assert np.array_equal(d_full.cpu().numpy()[lo:hi], d0)
    assert np.array_equal(p_full.cpu().numpy()[lo:hi], p0)


def test_many_near_ties():
    """Near ties under pressure: every third clip of a 5G + 37-clip batch is a near tie, so every
    workgroup of the fused kernel meets several of them, between clips whose next-clip loads are in
    flight.  Each is left DSP_CLIP_UNCERTIFIED by extract_kernel (and counted in queue_ws) and
    redone by extract_exact_kernel on the same stream: every clip must match the oracle and every
    near tie carry DSP_CLIP_FLAG_VAD_EXACT."""
    import torch
    from src.pipeline import FeatureExtractor, create_window
    from src.synth import make_batch
    G = grid()
    B = 5 * G + 37
    base = make_batch(64, base_seed=900)
    tie = near_tie_clip()
    clips = [tie if i % 3 == 0 else base[i % 64] for i in range(B)]
    off = np.zeros(B + 1, np.int64)
    off[1:] = np.cumsum([c.size for c in clips])
    pcm = torch.as_tensor(np.concatenate(clips + [np.zeros(8, np.int16)])).cuda()
    fx = FeatureExtractor(L, S, "hamming", True)
    out = {k: v.cpu().numpy() for k, v in fx(pcm, off).items()}
    _check(out, clips, create_window("hamming", L))
    assert ((out["status"][::3] >> 8) & 1).all(), "near ties were not redone exactly"
    assert not ((out["status"][1::3] >> 8) & 1).any()
