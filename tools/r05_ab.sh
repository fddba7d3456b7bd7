#!/bin/bash
# Round 5 GPU check: the GPU tests, then an A/B of extraction libraries with bench.py's own timing at
# 100k and 12.5k clips, then the phase stamps of the current build.
#   bash tools/r05_ab.sh TAG [variant...]   (variant: lib/libdsp_audiorec_<v>.so; base = current)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05a}; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
for clips in 100000 12500; do
  timeout -k 10 600 bash tools/ab_bench.sh $clips "$@" base 2>&1 | tee -a $O/ab.txt || exit 1
done
timeout -k 10 300 bash tools/stamps_seq.sh $T stamps > $O/stamps.txt 2>&1; tail -25 $O/stamps.txt
echo R05_DONE
