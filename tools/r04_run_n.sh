#!/bin/bash
# GPU tests, kernel-trace durations (r03 vs current), per-phase stamps (current vs r03)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04n}; mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 $R/gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 $R/gpurun_out/${T}_gpu_tests.log
bash tools/r04_kt.sh $T r03 base
bash tools/stamps_seq.sh $T stamps
