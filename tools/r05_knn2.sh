#!/bin/bash
# KNN GPU tests, A/B of KNN variants (bench_knn, both shapes), kernel stats of the current build,
# and the pilot sample sweep of the diagnostic build:  bash tools/r05_knn2.sh TAG "variants" "s0:s ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05k2}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_production.py -x -q --timeout 120 --timeout-method thread > $O/knn_tests.log 2>&1
rc=$?; tail -2 $O/knn_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/knn_tests.log | head; exit $rc; }
timeout -k 10 900 bash tools/r05_knn.sh $T $2 2>&1 | grep -E "nq=|DONE" | sed 's/"config".*"roofline"/../' | cut -c1-160
[ -n "$3" ] && timeout -k 10 600 bash tools/r05_knn_pilot.sh $3 | tee $O/pilot_sweep.txt
echo R05K2_DONE
