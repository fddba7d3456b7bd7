"""Diagnostics for the extraction kernel on the GPU box: flag rates and timings per variant."""
import os, sys, time, json
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dsp-audioreclabs_amd"))
import torch
from src.pipeline import FeatureExtractor
from src.synth import make_batch

def timeit(fx, x, reps=20):
    for _ in range(3): fx(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fx(x)
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps

C = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
STAMPS = "--stamps" in sys.argv
if STAMPS:
    import ctypes
    from src import _hip
    L_ = _hip.load_library()
    stamp_buf = torch.zeros((C, 16), dtype=torch.int64, device="cuda")
    L_.dsp_debug_set_stamp_buffer.argtypes = [ctypes.c_void_p]
    assert L_.dsp_debug_set_stamp_buffer(ctypes.c_void_p(stamp_buf.data_ptr())) == 0
x = torch.as_tensor(make_batch(C, base_seed=0)).cuda()
res = {}
for name, kw in [("vad_hamming", dict(window_type="hamming", do_endpoint_detection=True)),
                 ("novad_hamming", dict(window_type="hamming", do_endpoint_detection=False)),
                 ("vad_rect", dict(window_type="rectangular", do_endpoint_detection=True))]:
    fx = FeatureExtractor(1102, 441, **kw)
    out = fx(x)
    st = out["status"].cpu().numpy()
    ms = timeit(fx, x)
    if STAMPS:
        stamp_buf.zero_(); fx(x); torch.cuda.synchronize()
        st_ = stamp_buf.cpu().numpy().astype(np.float64)
        ph = {}
        seq = [0, 1, 2, 7, 8, 3, 4, 5, 9, 6]
        names = ["R1 load+stats", "R2a pos+chg", "R2b segments", "R3a vad frames", "R3 p90 rank",
                 "R3b scan", "R4 features", "R5 median ranks", "R5 stats+out"]
        for k in range(len(seq) - 1):
            a_, b_ = seq[k], seq[k + 1]
            ok = (st_[:, a_] > 0) & (st_[:, b_] > 0)
            if ok.any(): ph[names[k]] = float(np.median(st_[ok, b_] - st_[ok, a_]))
        # VAD off: stamps 7/8/3/4 missing -> bridge 2 -> 5 when absent
        if not ((st_[:, 7] > 0).any()):
            ok = (st_[:, 2] > 0) & (st_[:, 5] > 0)
            ph["R4 features (from R2a)"] = float(np.median(st_[ok, 5] - st_[ok, 2]))
        ok = (st_[:, 0] > 0) & (st_[:, 6] > 0)
        ph["total"] = float(np.median(st_[ok, 6] - st_[ok, 0]))
        # clip-to-clip period on one workgroup (includes the wait for the prefetched loads)
        G = 256
        if C > 2 * G:
            ph["period"] = float(np.median(st_[G:2 * G, 0] - st_[:G, 0]))
        span = (st_[:, 6].max() - st_[:, 0].min())
        ph["grid_span_cycles"] = float(span)
    res[name] = dict(ms=ms, flagged=int(((st >> 8) & 1).sum()), errors=int((st & 0xFF).astype(bool).sum()),
                     n_frames_mean=float(out["n_frames"].float().mean().item()))
    if STAMPS: res[name]["phase_cycles_median"] = ph
print(json.dumps(res, indent=1))
