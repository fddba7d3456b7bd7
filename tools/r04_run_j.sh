#!/bin/bash
# GPU tests, then kernel-trace durations of the headline bench: r03 library vs the current one
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04j}; mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 $R/gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 $R/gpurun_out/${T}_gpu_tests.log
bash tools/r04_kt.sh $T r03 base
