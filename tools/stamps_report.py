"""Summarise a raw stamp dump of tools/diag_extract.py (DIAG_SAVE): prologue, per-phase and
per-workgroup times in microseconds.  usage: stamps_report.py raw.npy [clock_ghz]"""
import sys
import numpy as np
st = np.load(sys.argv[1]).astype(np.float64)
G = int((st[:, 16] > 0).sum())
rt0, ck0, rt1, ck1 = (st[:G, k] for k in (16, 17, 22, 23))
ghz = np.median((ck1 - ck0) / (rt1 - rt0) * 0.1)
cyc = ghz * 1e3
C = len(st)
print("workgroups %d  clock %.3f GHz" % (G, ghz))
dur = (rt1 - rt0) / 100
print("wg us  p0 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(dur, [0, 50, 90, 100])))
# prologue, from the workgroup's own row (one clock): entry (17) -> window built (18) -> first
# clip claimed (19); clip rows are not the workgroup's (the queue hands out the first clip)
pro = (st[:G, 19] - ck0) / cyc
print("prologue us  p50 %.2f max %.2f  (window built p50 %.2f)" % (
    np.median(pro), pro.max(), np.median((st[:G, 18] - ck0) / cyc)))
tot = (st[:, 6] - st[:, 0]) / cyc
print("clip us  p50 %.2f p90 %.2f | first round p50 %.2f (wg<%d %.2f, wg>=%d %.2f) later %.2f" % (
    np.median(tot), np.percentile(tot, 90), np.median(tot[:G]), G // 2, np.median(tot[:G // 2]), G // 2,
    np.median(tot[G // 2:G]), np.median(tot[G:]) if C > G else 0))
names = {13: "R1 load wait", 1: "R1 stats", 2: "R2 pos", 7: "VAD pass A", 8: "VAD pass B", 3: "p90", 10: "noise+thr", 11: "scan",
         4: "vad out", 12: "R4 frames", 5: "R4 barrier(+issue)", 9: "R5 jobs", 6: "R5 out", 14: "end barrier",
         15: "flush"}
seq = [0, 13, 1, 2, 7, 8, 3, 10, 11, 4, 12, 5, 9, 6, 14, 15]
# loop top of each clip (slot 20): offsets load, its loads issued, queue claim -> clip start (0)
top = (st[:, 0] - st[:, 20]) / cyc
print("  %-14s p50 %.2f  (loop top -> clip start)" % ("loop top", np.median(top)))
# where the workgroups' time goes: prologue + the clips' spans (loop top -> flushed) against the
# workgroup's duration (the same shader clock)
span = (st[:, 15] - st[:, 20]) / cyc
wg_ck = (ck1 - ck0) / cyc
print("workgroup time: sum over workgroups %.0f us = prologue %.0f + clip spans %.0f + rest %.0f (per clip %.2f)" % (
    wg_ck.sum(), pro.sum(), span.sum(), wg_ck.sum() - pro.sum() - span.sum(), (wg_ck.sum() - pro.sum() - span.sum()) / C))
for a, b in zip(seq, seq[1:]):
    d = (st[:, b] - st[:, a]) / cyc
    print("  %-14s p50 %.2f  oldWG %.2f newWG %.2f" % (names[b], np.median(d), np.median(d[:G // 2]), np.median(d[G // 2:G])))

# per-wave load landing (slots 24..31, diagnostic build): time after the clip start, and the
# spread between the first and the last wave of the workgroup
if (st[:, 24:32] > 0).all(axis=1).any():
    ok = (st[:, 24:32] > 0).all(axis=1) & (st[:, 0] > 0)
    lw = (st[ok, 24:32] - st[ok, 0:1]) / cyc
    print("per-wave load landed after clip start us: median of max %.2f, median of min %.2f, per wave p50 %s" % (
        np.median(lw.max(1)), np.median(lw.min(1)), " ".join("%.2f" % v for v in np.median(lw, 0))))

# clip spans by the clip's ordinal in its workgroup (slot 21: the workgroup, diagnostic build) and
# the spread of the workgroups' clip counts
wg = st[:, 21].astype(np.int64)
if (st[:, 20] > 0).all() and wg.max() > 0:
    order = np.lexsort((st[:, 20], wg))
    ordinal = np.zeros(C, np.int64)
    w_sorted = wg[order]
    starts = np.r_[0, np.nonzero(np.diff(w_sorted))[0] + 1]
    for a, b in zip(starts, np.r_[starts[1:], C]):
        ordinal[order[a:b]] = np.arange(b - a)
    counts = np.bincount(wg, minlength=G)[:G]
    print("clips per workgroup: min %d p50 %d max %d" % (counts.min(), np.median(counts), counts.max()))
    for o in (0, 1, 2, 3, 5, 8, 12, 16, 24, 48, 96, 128):
        m = ordinal == o
        if m.sum() >= 16:
            print("  ordinal %3d: n %5d span mean %.2f p50 %.2f p90 %.2f us" % (o, m.sum(), span[m].mean(), np.median(span[m]),
                                                                        np.percentile(span[m], 90)))
    print("  span percentiles p50 %.2f p75 %.2f p90 %.2f p99 %.2f max %.2f" % tuple(np.percentile(span, [50, 75, 90, 99, 100])))
