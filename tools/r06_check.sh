#!/bin/bash
# Round 6 check after the KNN register-path changes (zscore fit one wave per column, re-rank and
# fallback with the query in registers): GPU tests, KNN merge-group A/B (KNN_MG 8 vs 16), KNN
# kernel stats at both shapes on extracted features, the re-read probe with its FETCH_SIZE pass,
# and the extraction at the N = 2 / N = 4 per-rank sizes:
#   bash tools/r06_check.sh TAG      (STEPS="tests knnab knn reread sizes" to choose)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r06g}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
S=${STEPS:-tests knnab knn reread sizes}
if [[ " $S " == *" tests "* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [[ " $S " == *" knnab "* ]]; then
  bash tools/knn_libs_ab.sh base mg16 base mg16 > $O/knn_ab.txt 2>&1 || { cat $O/knn_ab.txt; exit 1; }
  cat $O/knn_ab.txt
fi
if [[ " $S " == *" knn "* ]]; then
  for q in 12500 100000; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/knn_$q -o kt -- python3 $R/tools/bench_knn.py --queries $q --no-cpu --graph > $O/knn_$q.json 2> $O/knn_$q.err) || { tail -5 $O/knn_$q.err; exit 1; }
    tail -1 $O/knn_$q.json | cut -c1-300
  done
fi
if [[ " $S " == *" reread "* ]]; then
  timeout -k 10 200 python3 tools/probe_reread.py > $O/reread.json 2> $O/reread.err || { tail -5 $O/reread.err; exit 1; }
  tail -1 $O/reread.json
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/reread_pmc -o pmc -- python3 $R/tools/probe_reread.py > $O/reread_pmc.json 2> $O/reread_pmc.err) || { tail -5 $O/reread_pmc.err; exit 1; }
fi
if [[ " $S " == *" sizes "* ]]; then
  for c in 50000 25000; do bash tools/ab_bench.sh $c base >> $O/sizes.txt 2>&1 || { tail -5 $O/sizes.txt; exit 1; }; done
  cat $O/sizes.txt
fi
echo R06G_DONE
