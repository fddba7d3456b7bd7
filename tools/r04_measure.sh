#!/bin/bash
# Round-4 measurement on the GPU box (via gpurun): the lane-exchange check, GPU tests, the bench
# line with rocprofv3 kernel stats and FETCH/WRITE PMC (tools/profile_round.sh), KNN kernel stats
# at the per-rank and the full shape.  Every GPU step has its own time limit; the first failure
# ends the script (set -e).
# usage: bash tools/r04_measure.sh TAG [--no-tests] [--no-knn]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04a}; shift || true
O=$R/gpurun_out/$T; mkdir -p $O; cd $R
TESTS=1; KNN=1
for a in "$@"; do case $a in --no-tests) TESTS=0;; --no-knn) KNN=0;; esac; done
if [ -x tools/ubench/perm_check ]; then timeout -k 10 60 tools/ubench/perm_check | tee $O/perm_check.txt; fi
if [ $TESTS = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
fi
bash tools/profile_round.sh $T
export TMPDIR=/tmp
if [ $KNN = 1 ]; then
  for nq in 12500 100000; do
    timeout -k 10 200 python3 tools/bench_knn.py --no-cpu --queries $nq > $O/knn_$nq.json
    cat $O/knn_$nq.json
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/knn_kt_$nq -o kt -- python3 $R/tools/bench_knn.py --no-cpu --queries $nq > $O/knn_kt_$nq.log 2>&1)
  done
fi
echo MEASURE_DONE
