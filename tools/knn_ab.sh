#!/bin/bash
# KNN A/B on the GPU box: parity tests, then bench_knn (12.5k shard and 100k queries x 100k refs)
# plus kernel stats
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_dropin.py tests/test_gpu_dataset.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gtk.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gtk.log; [ $rc -ne 0 ] && exit 1
run() { timeout -k 10 200 python3 tools/bench_knn.py --no-cpu "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['queries'], d['ms'], d['roofline']['frac'])"; }
echo -n "shard: "; run
echo -n "full:  "; run --queries 100000
for Q in 12500 100000; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/knnkt_$Q -o kt -- python3 tools/bench_knn.py --no-cpu --queries $Q > /dev/null 2>&1
  python3 - gpurun_out/knnkt_$Q <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "knn" in r["Name"]: print("  %-40s calls %4s avg_us %9.1f" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
