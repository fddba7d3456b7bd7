#!/bin/bash
# 2-rank rehearsal of bench.py on one GPU (gloo; value = extraction + all-gather, plus
# value_extract_only) at the configs[3] size, then the f4 end-to-end breakdown of run.py
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05m}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
DSP_BENCH_ONE_DEVICE=1 DSP_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 --sweep-clips 0 --knn-ref 0 --no-cpu --small-clips 0 --no-cfg0 > $O/rehearsal.json 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
tail -1 $O/rehearsal.json
timeout -k 10 400 python3 tools/f4_breakdown.py --files 2000 > $O/f4.json 2> $O/f4.err || { tail -30 $O/f4.err; exit 1; }
tail -1 $O/f4.json
echo R05M_DONE
