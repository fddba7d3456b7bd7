#!/usr/bin/env python3
"""Average duration of the dispatches of bench.py's TIMED steps in a rocprofv3 kernel trace.

    python tools/kt_timed_avg.py <kt_kernel_trace.csv> [K=20] [kernel=extract_kernel<true>]

bench.py's order of extraction dispatches (profile_round.sh flags: no sweep / KNN / configs legs):
first launches and isolated timed launches, the capture stream's first launch, the graph's first
replay (K), the TIMED replay (K), then one launch into fresh buffers (the timed-output check).  The
timed dispatches are therefore the K before the last one.  Prints the kernel's mean over them, over
all dispatches (what --stats reports), and the timed span per step (first start to last end / K,
which includes the exact kernel and the launch gaps, as bench.py's HIP events do).
"""
import csv
import statistics
import sys

path = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
name = sys.argv[3] if len(sys.argv) > 3 else "extract_kernel<true>"
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
timed = rows[-(K + 1):-1]
td = dur[-(K + 1):-1]
span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e6 / K
print("dispatches %d; timed %d: mean %.4f ms (min %.4f, max %.4f); all: mean %.4f ms; timed span per step %.4f ms"
      % (len(dur), len(td), statistics.mean(td), min(td), max(td), statistics.mean(dur), span))
