"""Per-phase cost by doubling (diagnostic build, DSP_LIB_PATH = libdsp_audiorec_stamps.so): each
idempotent phase runs twice in turn; the extra kernel time is the phase's own marginal cost with
the rest of the clip unchanged.  usage: double.py [clips]"""
import ctypes, json, os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "dsp-audioreclabs_amd"))
import torch
from src import _hip
from src.pipeline import FeatureExtractor
from src.synth import make_batch
L_ = _hip.load_library()
L_.dsp_debug_set_skip.argtypes = [ctypes.c_int]
C = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
x = torch.as_tensor(make_batch(C, base_seed=0)).cuda()
fx = FeatureExtractor(1102, 441, "hamming", True)
PH = {1: "R1", 2: "R2", 4: "VAD frames", 128: "VAD pass A", 8: "p90", 16: "scan", 32: "R4", 64: "R5"}
def t(mask, reps=40):
    L_.dsp_debug_set_skip(mask)
    for _ in range(3): fx(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fx(x)
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
ref = fx(x)["feat"].clone()
base = [t(0) for _ in range(3)]
res = {"base_us": round(min(base), 2)}
for bit, nm in PH.items():
    v = min(t(bit << 8) for _ in range(2))
    out = fx(x)["feat"]
    same = bool(torch.equal(out.nan_to_num(0), ref.nan_to_num(0)))
    res[nm] = {"us": round(v, 2), "phase_us": round(v - res["base_us"], 2), "results_unchanged": same}
L_.dsp_debug_set_skip(0)
print(json.dumps(res, indent=1))
