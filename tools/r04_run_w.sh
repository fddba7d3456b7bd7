#!/bin/bash
# GPU tests, then the headline profile at 100k and 12.5k clips (bench line, kernel stats,
# FETCH/WRITE PMC) and the phase stamps
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04w}; mkdir -p $R/gpurun_out; cd $R; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
bash tools/profile_round.sh $T
bash tools/profile_round.sh ${T}_12k --clips 12500 --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0
bash tools/stamps_seq.sh $T stamps
rm -f gpurun_out/st_${T}_stamps/*.npy
