"""Summarise a stamp dump of the pipelined fused kernel (make stamps; tools/diag_extract.py with
DIAG_SAVE): per trip of a workgroup's loop (one trip per clip B entering), the four stages and the
single-wave phases, in microseconds.  usage: stamps_pipe.py raw.npy"""
import sys
import numpy as np
st = np.load(sys.argv[1]).astype(np.float64)
G = int((st[:, 16] > 0).sum())
rt0, ck0, rt1, ck1 = (st[:G, k] for k in (16, 17, 22, 23))
ghz = np.median((ck1 - ck0) / (rt1 - rt0) * 0.1)
cyc = ghz * 1e3
print("workgroups %d  clock %.3f GHz  kernel (wg p50) %.1f us" % (G, ghz, np.median((rt1 - rt0) / 100)))
ok = (st[:, 0] > 0) & (st[:, 3] > 0)
t = st[ok]
def d(a, b):
    x = (t[:, b] - t[:, a]) / cyc
    return x[(t[:, a] > 0) & (t[:, b] > 0)]
for nm, a, b in (("trip (S1..S4)", 0, 3), ("S1 R1(B) | scan(A)", 0, 1), ("  scan(A), wave 0", 0, 11),
                 ("S2 R2(B), crop(A)", 1, 2), ("S3 VAD(B) + R4(A), wave 0", 2, 14), ("S3 ... wave 7", 2, 12),
                 ("S4 R5(A) | p90(B)", 14, 3), ("  R5 job, wave 0", 14, 15), ("  p90(B), wave 6", 14, 8)):
    x = d(a, b)
    if x.size:
        print("  %-28s p50 %6.2f  p10 %6.2f  p90 %6.2f" % (nm, np.median(x), np.percentile(x, 10), np.percentile(x, 90)))
# per-CU clip interval: trips per workgroup over its lifetime
dur = (rt1 - rt0) / 100
trips = ok.sum()
print("clips stamped %d; workgroup lifetime p50 %.1f us -> %.2f us per clip per workgroup, %.2f per CU (2 WG/CU)" % (
    trips, np.median(dur), np.median(dur) * G / max(trips, 1), np.median(dur) * G / max(trips, 1) / 2))
