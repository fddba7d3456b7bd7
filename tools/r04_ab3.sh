#!/bin/bash
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04f}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/ab_bench.sh 100000 r03 base seq2 > $O/ab100k.txt 2>&1; cat $O/ab100k.txt
bash tools/pmc_insts_var.sh ${T}_pmc base seq2
echo DONE
