#!/bin/bash
# Round-3 measurement pass on the GPU box: GPU tests, the misaligned-load probe, phase stamps at
# 100 000 clips, then tools/profile_round.sh (bench line, kernel stats, FETCH/WRITE PMC).
# usage (via gpurun): bash tools/r03_measure.sh TAG [skip-tests]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r03a}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -2 $O/gpu_tests.log
fi
if [ -x tools/ubench/misalign ]; then timeout -k 10 60 tools/ubench/misalign > $O/misalign.txt 2>&1; cat $O/misalign.txt; fi
if [ -f dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so ]; then bash tools/stamps_seq.sh $T stamps | head -30; fi
bash tools/profile_round.sh $T
