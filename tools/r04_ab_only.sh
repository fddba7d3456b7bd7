set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=r04b; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
bash tools/ab_bench.sh 100000 r03 pipe1 base > $O/ab100k.txt 2>&1; cat $O/ab100k.txt
for nq in 12500 100000; do
  timeout -k 10 200 python3 tools/bench_knn.py --no-cpu --queries $nq > $O/knn_$nq.json; cat $O/knn_$nq.json
done
bash tools/stamps_run.sh $T 100000 || true
echo DONE
