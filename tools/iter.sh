#!/bin/bash
# One GPU iteration during kernel work: the GPU test suite, then an A/B of library variants with
# bench.py's workload.  usage: tools/iter.sh [--no-tests] NAME... [-- extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "$1" = "--no-tests" ]; then shift; else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/iter_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|^E " gpurun_out/iter_tests.log | head -30; exit $rc; }
fi
bash tools/abbench.sh "$@"
