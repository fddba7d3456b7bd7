#!/bin/bash
# Round-4 A/B on the GPU box: lane-exchange check, GPU tests, then extraction A/B of the round-3
# library (lib/libdsp_audiorec_r03.so, built from git history) against the current one, and the
# KNN job at both shapes.  usage: bash tools/r04_ab.sh TAG [--no-tests]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04b}; shift || true
O=$R/gpurun_out/$T; mkdir -p $O; cd $R
TESTS=1; for a in "$@"; do case $a in --no-tests) TESTS=0;; esac; done
timeout -k 10 60 tools/ubench/perm_check | tee $O/perm_check.txt
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
bash tools/ab_bench.sh 100000 r03 pipe1 base > $O/ab100k.txt 2>&1; cat $O/ab100k.txt
for nq in 12500 100000; do
  timeout -k 10 200 python3 tools/bench_knn.py --no-cpu --queries $nq > $O/knn_$nq.json; cat $O/knn_$nq.json
done
bash tools/stamps_run.sh $T 100000 || true
echo DONE
