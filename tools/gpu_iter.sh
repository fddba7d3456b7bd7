#!/bin/bash
# one GPU iteration: GPU tests, then a rocprofv3 kernel-trace of the 100k-clip bench (stats to
# gpurun_out/$1/), then the plain bench line.  usage: tools/gpu_iter.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-it}; shift || true
O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -20; exit $rc; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --steps 10 "$@" > $O/kt_bench.json 2> $O/kt.err || exit 1
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "dsp::" in r["Name"]:
        print("%-60s calls %5s avg_us %10.1f" % (r["Name"].replace("void ", "")[:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
cd $R
timeout -k 10 300 python3 bench.py --no-cpu --knn-ref 0 --sweep-clips 0 "$@" > $O/bench.json && python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', d['value'], 'kernel_ms', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'])"
