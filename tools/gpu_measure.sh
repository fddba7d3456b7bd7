set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r1; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --knn-ref 0 --sweep-clips 0 > $O/b100k.json 2> $O/b100k.err
timeout -k 10 300 python bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --clips 12500 > $O/b12k.json 2> $O/b12k.err
timeout -k 10 300 python bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --clips 1000 > $O/b1k.json 2> $O/b1k.err
cat $O/b100k.json $O/b12k.json $O/b1k.json
tail -3 $O/gpu_tests.log
