#!/bin/bash
# Round-3 final measurement on the GPU box: GPU tests, the bench line with rocprofv3 kernel stats
# and FETCH/WRITE PMC (tools/profile_round.sh), and KNN kernel stats at the per-rank and full shape.
# usage (via gpurun): bash tools/r03_final.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r03b}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
bash tools/profile_round.sh $T
export TMPDIR=/tmp
for nq in 12500 100000; do
  timeout -k 10 200 python3 tools/bench_knn.py --no-cpu --queries $nq > $O/knn_$nq.json
  cat $O/knn_$nq.json
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/knn_kt_$nq -o kt -- python3 $R/tools/bench_knn.py --no-cpu --queries $nq > $O/knn_kt_$nq.log 2>&1)
done
echo FINAL_DONE
