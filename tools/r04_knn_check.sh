#!/bin/bash
# KNN GPU tests (and the suites that run the KNN), the bench at both shapes, and optionally a forced
# split sweep at the rank shape: bash tools/r04_knn_check.sh [split...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_production.py tests/test_gpu_dataset.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/knn_tests.log 2>&1 || { tail -30 gpurun_out/knn_tests.log; exit 1; }
tail -1 gpurun_out/knn_tests.log
for nq in 12500 100000; do timeout -k 10 200 python3 tools/bench_knn.py --no-cpu --queries $nq; done
[ $# -gt 0 ] && bash tools/knn_split_sweep.sh 12500 "$@"
exit 0
