#!/bin/bash
# Runs on the GPU box (via gpurun): the full bench line, then rocprofv3 kernel trace/stats and the
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) of the headline extraction alone (no window
# sweep, KNN leg or CPU baseline, so the extract_kernel averages are the headline's launches).
# Usage: tools/profile_round.sh <tag> [extra bench args]
set -e
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python3 $R/bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
H="--no-cpu --sweep-clips 0 --knn-ref 0 --no-cfg0 --small-clips 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py $H "$@" > $OUT/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $R/bench.py $H --steps 8 --warmup 1 "$@" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 $R/bench.py $H --steps 8 --warmup 1 "$@" > $OUT/pmc_write.log 2>&1
echo PROFILE_DONE
