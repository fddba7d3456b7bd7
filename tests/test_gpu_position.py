"""Per-clip results do not depend on where a clip sits in the packed buffer, nor on which kernel
processed it.  Both extraction kernels sum the windowed frames in one canonical order defined in
clip coordinates (csrc/dsp_device.h), so:
  * the same clips packed at leads 0..7 (every alignment of a clip's first sample to the 16-B
    vectors of the buffer) give bit-identical feat / seq / start_end / n_frames / status;
  * dsp_extract_general (global-memory kernel) and dsp_extract_features (fused) give the same bits;
  * extraction over shard_range blocks concatenates to the single launch for any shard size
    (gather(shards) == single-GPU output), e.g. B = 6001 over 8 ranks.
The reference computes per file (experiments/run_experiments.py:82-111): a clip's features are a
function of the clip alone.
"""
import numpy as np
import pytest

import oracle
from test_gpu_extract import feat_close

pytestmark = pytest.mark.gpu

L, S = 1102, 441


def _clips():
    """1 s clips plus lengths that end on / off vector boundaries at every lead (the odd-lead
    clip whose last sample sits in a straddling dword), short and padded-tail clips."""
    from src.synth import make_clip
    lens = [44100, 44100, 44099, 44097, 40001, 30007, 22050, 8191, 5000, 1500, 1103, 1102, 700, 44095,
            44093, 44091, 44089, 12345, 20001, 44100 - 3]
    return [make_clip(7000 + i, n) for i, n in enumerate(lens)]


def _pack(clips, lead):
    """Pack clips back to back after `lead` junk samples: every clip moves by `lead` samples."""
    parts = [np.full(lead, 1234, np.int16)] + list(clips) + [np.zeros(16, np.int16)]
    off = np.zeros(len(clips) + 1, np.int64)
    off[0] = lead
    off[1:] = lead + np.cumsum([len(c) for c in clips])
    return np.concatenate(parts), off


def _run(fx, pcm, off):
    import torch
    o = fx(torch.as_tensor(pcm).cuda(), off)
    return {k: v.cpu().numpy().copy() for k, v in o.items()}


@pytest.mark.parametrize("win,vad", [("hamming", True), ("hanning", False), ("rectangular", True)])
def test_leads_bit_identical(win, vad):
    from src.pipeline import FeatureExtractor
    clips = _clips()
    fx = FeatureExtractor(L, S, win, vad, return_sequences=True, return_vad_lists=True)
    base = None
    for lead in range(8):
        pcm, off = _pack(clips, lead)
        out = _run(fx, pcm, off)
        assert not (out["status"] & 0xFF).any()
        if base is None:
            base = out
            from src.pipeline import create_window
            w = create_window(win, L)
            for i, c in enumerate(clips):  # and the oracle, once
                r = oracle.process_clip(c, L, S, w, do_vad=vad)
                assert tuple(out["start_end"][i]) == (r["start"], r["end"]), i
                assert not feat_close(out["feat"][i], r["feat"]).any(), i
            continue
        for k in base:
            assert np.array_equal(base[k], out[k]), (lead, k)


def test_general_equals_fused_bitwise():
    """dsp_extract_general on clips the fused kernel also takes: the same bits."""
    from src.pipeline import FeatureExtractor
    from test_gpu_general import _general
    clips = _clips()
    pcm, off = _pack(clips, 3)
    for win, vad in (("hamming", True), ("hanning", True), ("rectangular", False)):
        fx = FeatureExtractor(L, S, win, vad, return_sequences=True)
        a = _run(fx, pcm, off)
        b = _general(pcm, off, L, S, win, vad)
        for k in ("feat", "start_end", "n_frames", "status"):
            assert np.array_equal(a[k], b[k]), (win, vad, k)
        F = a["n_frames"]
        for i in range(len(clips)):
            assert np.array_equal(a["seq"][i, :F[i]], b["seq"][i, :F[i]]), (win, vad, i)


def test_sharded_extraction_odd_shard_size():
    """8 simulated ranks over B = 6001 clips (blocks of 751 / 750: every rank after the first
    starts at a different lead): the concatenation equals the single launch bit for bit."""
    import torch
    from src.distributed import shard_range
    from src.pipeline import FeatureExtractor
    from src.synth import make_batch_device
    B, P = 6001, 8
    x = make_batch_device(B, "cuda", base_seed=21)
    flat = x.reshape(-1)
    off = torch.arange(B + 1, dtype=torch.int64, device="cuda") * x.shape[1]
    fx = FeatureExtractor(L, S, "hamming", True)
    full = {k: v.clone() for k, v in fx(flat, off).items()}
    parts = []
    for r in range(P):
        lo, hi = shard_range(B, r, P)
        # each rank packs only its block: the block's first clip lands at the rank's own lead
        sub = flat[lo * x.shape[1]:hi * x.shape[1]].clone()
        o = torch.arange(hi - lo + 1, dtype=torch.int64, device="cuda") * x.shape[1]
        parts.append({k: v.clone() for k, v in fx(sub, o).items()})
    for k in full:
        assert torch.equal(torch.cat([p_[k] for p_ in parts]), full[k]), k
    # and a shifted copy of the whole batch (lead 5): same bits
    shifted = torch.cat([torch.zeros(5, dtype=torch.int16, device="cuda"), flat, torch.zeros(8, dtype=torch.int16, device="cuda")])
    sh = fx(shifted, off + 5)
    for k in full:
        assert torch.equal(sh[k], full[k]), k


def test_two_streams_concurrent_and_static_split():
    """Two extractions in flight at once on two streams -- two extractors, and ONE extractor
    launching on both streams with no sync in between (its clip-queue scratch is per stream, so
    neither launch can claim the other's chunks) -- and the C ABI's static split (queue_ws =
    NULL): every result equals the oracle / the queued launch bit for bit."""
    import torch
    from src import _hip
    from src.pipeline import FeatureExtractor, create_window
    from src.synth import make_batch
    xa = torch.as_tensor(make_batch(3000, base_seed=31)).cuda()
    xb = torch.as_tensor(make_batch(2500, base_seed=77, n_samples=30000)).cuda()
    fa = FeatureExtractor(L, S, "hamming", True)
    fb = FeatureExtractor(1024, 512, "hanning", True)
    ref_a = {k: v.clone() for k, v in fa(xa).items()}
    ref_b = {k: v.clone() for k, v in fb(xb).items()}
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(5):
        with torch.cuda.stream(sa):
            oa = fa(xa)
        with torch.cuda.stream(sb):
            ob = fb(xb)
        torch.cuda.synchronize()
        for k in ref_a:
            assert torch.equal(oa[k], ref_a[k]), k
            assert torch.equal(ob[k], ref_b[k]), k
    # one extractor, two streams, batches of two sizes (separate output buffers) in flight at once
    xc = xa[:2300].contiguous()
    ref_c = {k: v.clone() for k, v in fa(xc).items()}
    for _ in range(5):
        with torch.cuda.stream(sa):
            oa = fa(xa)
        with torch.cuda.stream(sb):
            oc = fa(xc)
        torch.cuda.synchronize()
        for k in ref_a:
            assert torch.equal(oa[k], ref_a[k]), k
            assert torch.equal(oc[k], ref_c[k]), k
    for k in ref_c:
        assert torch.equal(ref_c[k], ref_a[k][:2300]), k
    host = xa.cpu().numpy()
    for i in range(0, 3000, 211):
        r = oracle.process_clip(host[i], L, S, create_window("hamming", L))
        assert tuple(ref_a["start_end"][i].tolist()) == (r["start"], r["end"])
        assert not feat_close(ref_a["feat"][i].cpu().numpy(), r["feat"]).any()
    # queue_ws = NULL: the static split, same bits, into four separate arrays (out_stride 0)
    out = {k: torch.empty_like(v) for k, v in ref_a.items() if k != "rows"}
    flat = xa.reshape(-1)
    off = torch.arange(3001, dtype=torch.int64, device="cuda") * xa.shape[1]
    P = _hip.ptr
    rc = _hip.lib().dsp_extract_features(P(flat), P(off), 3000, xa.shape[1], L, S, P(fa.window), 1, 0.5, 0.1, 1.5,
                                         P(out["feat"]), P(out["start_end"]), P(out["n_frames"]), P(out["status"]),
                                         0, None, None, 0, None, 0, None, _hip.stream_handle())
    _hip.check(rc, "dsp_extract_features")
    torch.cuda.synchronize()
    for k in out:
        assert torch.equal(out[k], ref_a[k]), k


@pytest.mark.gpu
def test_queue_modes_same_bits():
    """Every clip-queue mode gives the static split's bits: 1 000 clips (<= 1.5 per workgroup: the
    static split), 1 400 (1-clip claimed chunks), 4 000 (2-clip chunks), and each against the
    C ABI's queue_ws = NULL launch of the same clips."""
    import torch
    from src import _hip
    from src.pipeline import FeatureExtractor
    from src.synth import make_batch
    fx = FeatureExtractor(L, S, "hamming", True)
    for B in (1000, 1400, 4000):
        x = torch.as_tensor(make_batch(B, base_seed=900 + B)).cuda()
        ref = {k: v.clone() for k, v in fx(x).items()}
        out = {k: torch.empty_like(v) for k, v in ref.items() if k != "rows"}
        flat = x.reshape(-1)
        off = torch.arange(B + 1, dtype=torch.int64, device="cuda") * x.shape[1]
        P = _hip.ptr
        rc = _hip.lib().dsp_extract_features(P(flat), P(off), B, x.shape[1], L, S, P(fx.window), 1, 0.5, 0.1, 1.5,
                                             P(out["feat"]), P(out["start_end"]), P(out["n_frames"]),
                                             P(out["status"]), 0, None, None, 0, None, 0, None, _hip.stream_handle())
        _hip.check(rc, "dsp_extract_features")
        torch.cuda.synchronize()
        for k in out:
            assert torch.equal(out[k], ref[k]), (B, k)
