import ctypes, os, sys, numpy as np
os.environ["DSP_LIB_PATH"] = os.path.abspath("dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so")
sys.path[:0] = ["dsp-audioreclabs_amd", "oracle"]
import torch
import oracle
from src import _hip
from src.pipeline import FeatureExtractor, create_window
from src.synth import make_clip
Lb = _hip.load_library()
dump = torch.zeros((2, 4096), dtype=torch.int32, device="cuda")
Lb.dsp_debug_set_dump_buffer.argtypes = [ctypes.c_void_p]
assert Lb.dsp_debug_set_dump_buffer(ctypes.c_void_p(dump.data_ptr())) == 0
base = make_clip(60, 44100)
fx = FeatureExtractor(1102, 441, "hamming", False, return_sequences=True)
for n, lead, last in ((3000, 5, -300), (2000, 0, -300), (44100, 0, 300)):
    c = base[:n].copy(); c[-1] = last
    off = np.array([0, lead, lead + n], np.int64)
    pcm = np.concatenate([np.zeros(lead, np.int16), c, np.zeros(8, np.int16)])
    out = {k: v.cpu().numpy() for k, v in fx(torch.as_tensor(pcm).cuda(), off).items()}
    d = dump[1].cpu().numpy().view(np.uint32)
    k = c.astype(np.int64); mq = k.sum() / n; tpos = int(np.floor(mq)) + 1
    pos = (k >= tpos).astype(np.uint8)
    chg = np.zeros(4096 * 32, np.uint8)
    chg[lead:lead + n - 1] = pos[:-1] ^ pos[1:]
    bits = np.unpackbits(d.view(np.uint8), bitorder="little")
    nw = ((lead + n + 7) // 8 + 3) // 4
    diff = np.nonzero(bits[:nw * 32] != chg[:nw * 32])[0]
    print(n, lead, last, "nw", nw, "diff bits", diff[:20], "total", len(diff), "tail words", [hex(x) for x in d[nw - 2:nw + 3]])
