#!/bin/bash
# GPU tests on the product library, then an A/B of library variants at 100k clips:
#   tools/gpu_ab.sh TAG variant...   (lib/libdsp_audiorec_<variant>.so; "base" = the product library)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|^E " $O/gpu_tests.log | head -30; exit $rc; }
bash tools/ab_bench.sh 100000 base "$@"
