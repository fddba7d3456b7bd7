#!/bin/bash
# Round-2 measurement call: GPU tests, profile_round.sh at the headline 100k clips (full bench
# line: window sweep, KNN leg, CPU baseline) and at 12.5k clips (the per-GPU share at N=8), then
# the KNN kernel stats.  usage: tools/r02_measure.sh TAG_100K TAG_12K
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r02m; mkdir -p $O; cd $R
A=${1:-r02a}; B=${2:-r02b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/gpu_tests.log 2>&1 \
  || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/profile_round.sh $A && bash tools/profile_round.sh $B --clips 12500 --knn-ref 12500 --cpu-seconds 5 && bash tools/knn_ab.sh
