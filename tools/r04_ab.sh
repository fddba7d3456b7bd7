set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04b; mkdir -p $O; cd $R
timeout -k 10 60 tools/ubench/perm_check | tee $O/perm_check.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/ab_bench.sh 100000 r03 base > $O/ab100k.txt 2>&1; cat $O/ab100k.txt
bash tools/ab_bench.sh 12500 r03 base > $O/ab12k.txt 2>&1; cat $O/ab12k.txt
echo DONE
