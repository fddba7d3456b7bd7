#!/bin/bash
# Runs on the GPU box (via gpurun): bench + rocprofv3 kernel trace/stats + PMC passes.
# Usage: tools/profile_round.sh <tag> [extra bench args]
set -e
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 $R/bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --no-cpu "$@" > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $R/bench.py --no-cpu --steps 8 --warmup 1 "$@" > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 $R/bench.py --no-cpu --steps 8 --warmup 1 "$@" > $OUT/pmc_write.log 2>&1
echo PROFILE_DONE
