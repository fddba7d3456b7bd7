#!/bin/bash
# round 6: GPU tests (TESTS=1, default on), then the default bench line (BENCH=1), optionally the
# rocprofv3 kernel-trace of the headline launch (PROF=1):  bash tools/r06_run.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r06}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -30; exit $rc; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 3000 $O/bench.json
fi
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 20 > $O/prof_bench.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
  find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv; head -5 $O/kernel_stats.csv
fi
echo R06RUN_DONE
