"""Phase ablation timing (diagnostic build): kernel time with each phase skipped.
DSP_LIB_PATH must point at libdsp_audiorec_stamps.so."""
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
vad = "--novad" not in sys.argv
x = torch.as_tensor(make_batch(C, base_seed=0)).cuda()
fx = FeatureExtractor(1102, 441, "hamming", vad)
def t(mask, reps=30):
    L_.dsp_debug_set_skip(mask)
    for _ in range(3): fx(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fx(x)
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
names = {0: "none", 4: "scan", 4 | 2: "scan+p90", 4 | 2 | 1: "scan+p90+vad frames", 8: "R4",
         16: "R5 ranks", 32: "R5 stats", 16 | 32: "R5", 64: "R2 bits", 8 | 16 | 32: "R4+R5",
         255 & ~128: "all but R1", 255: "everything"}
if "--once" in sys.argv:  # one configuration (DSP_SKIP) for PMC collection
    t(int(os.environ.get("DSP_SKIP", "0")), reps=5)
    sys.exit(0)
base = t(0)
res = {"base_us": round(base, 2)}
for m, nm in names.items():
    if m == 0: continue
    v = t(m)
    res[nm] = {"us": round(v, 2), "saved_us": round(base - v, 2)}
L_.dsp_debug_set_skip(0)
print(json.dumps(res, indent=1))
