#!/bin/bash
# Round 6 record: GPU tests, smoke(), the headline profile at 100k / 12.5k / 1 000 clips
# (profile_round.sh: bench line, kernel trace, FETCH/WRITE PMC passes), the instruction mix and
# busy counters at 100k, the 2-rank gloo rehearsal, KNN kernel stats at both shapes on extracted
# features:  bash tools/r06_final.sh TAG      (STEPS="tests prof pmc rehearsal knn" to choose)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r06f}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
S=${STEPS:-tests prof pmc rehearsal knn}
if [[ " $S " == *" counters "* ]]; then  # which memory-side counters this gfx950 exposes (MALL / DRAM)
  (cd /tmp && timeout -k 10 120 rocprofv3 -L > $O/counters_all.txt 2>&1); grep -i -E "mall|dram|EA0_RD|EA_RD|tcc_ea" $O/counters_all.txt | head -60 > $O/counters_mem.txt; wc -l $O/counters_mem.txt
fi
if [[ " $S " == *" tests "* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [[ " $S " == *" prof "* ]]; then
  bash tools/profile_round.sh ${T}p > /dev/null 2>&1 && bash tools/profile_round.sh ${T}p12 --clips 12500 > /dev/null 2>&1 && \
    bash tools/profile_round.sh ${T}p1k --clips 1000 > /dev/null 2>&1 || { echo "profile_round failed"; exit 1; }
  tail -1 $O/../${T}p/bench.json | cut -c1-600
fi
if [[ " $S " == *" pmc "* ]]; then
  bash tools/r05_pmc2.sh ${T}pmc base > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
  cat $O/../${T}pmc/pmc.txt $O/../${T}pmc/pmc_busy.txt 2>/dev/null | head -40
fi
if [[ " $S " == *" rehearsal "* ]]; then
  DSP_BENCH_ONE_DEVICE=1 DSP_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 2 --sweep-clips 0 --knn-ref 20000 --no-cpu --small-clips 0 --no-cfg0 > $O/rehearsal.json 2> $O/rehearsal.err || { tail -5 $O/rehearsal.err; exit 1; }
  tail -1 $O/rehearsal.json | cut -c1-400
fi
if [[ " $S " == *" knn "* ]]; then
  for q in 12500 100000; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/knn_$q -o kt -- python3 $R/tools/bench_knn.py --queries $q --no-cpu --graph > $O/knn_$q.json 2> $O/knn_$q.err) || { tail -5 $O/knn_$q.err; exit 1; }
    tail -1 $O/knn_$q.json | cut -c1-300
  done
fi
echo R06F_DONE
