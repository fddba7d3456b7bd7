#!/bin/bash
# GPU tests, KNN bench at both shapes, the 2-rank rehearsal of bench.py on one GPU, and the
# instruction mix of the phase ablations (DSP_ABL builds: outputs wrong, counts only)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04t}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for nq in 12500 100000; do timeout -k 10 200 python3 tools/bench_knn.py --queries $nq > $O/knn_$nq.json 2> $O/knn_$nq.err; cat $O/knn_$nq.json; done
DSP_BENCH_ONE_DEVICE=1 DSP_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --clips 20001 --sweep-clips 2000 --knn-ref 20000 --no-cpu --small-clips 0 --no-cfg0 > $O/rehearsal.json 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
tail -1 $O/rehearsal.json
bash tools/pmc_insts_var.sh ${T}_pmc base abl1 abl2 abl4 abl8
