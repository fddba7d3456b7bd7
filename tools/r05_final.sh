#!/bin/bash
# Round 5 final record: GPU tests, smoke(), the headline profile at 100k / 12.5k / 1 000 clips
# (profile_round.sh), the 2-rank gloo rehearsal, KNN kernel stats at both shapes
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05f}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1; tail -1 $O/smoke.log
bash tools/profile_round.sh ${T}p > /dev/null 2>&1 && bash tools/profile_round.sh ${T}p12 --clips 12500 > /dev/null 2>&1 && bash tools/profile_round.sh ${T}p1k --clips 1000 > /dev/null 2>&1 || exit 1
tail -1 $O/../${T}p/bench.json | cut -c1-400
DSP_BENCH_ONE_DEVICE=1 DSP_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 --sweep-clips 0 --knn-ref 0 --no-cpu --small-clips 0 --no-cfg0 > $O/rehearsal.json 2> $O/rehearsal.err || { tail -5 $O/rehearsal.err; exit 1; }
tail -1 $O/rehearsal.json | cut -c1-300
echo R05F_DONE
