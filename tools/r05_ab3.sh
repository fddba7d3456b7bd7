#!/bin/bash
# GPU tests (optional, TESTS=1), then an A/B of library variants at the clip counts in $CLIPS
# (default 100000 12500 1000):  bash tools/r05_ab3.sh TAG "v1 v2 ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05z}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
fi
for clips in ${CLIPS:-100000 12500 1000}; do
  timeout -k 10 600 bash tools/ab_bench.sh $clips $2 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt || exit 1
done
echo R05AB3_DONE
