#!/bin/bash
# quick GPU check of the working tree: GPU tests (stop at first failure) + headline bench
# usage (via gpurun): bash tools/quick_gpu.sh TAG [pytest -k expr]
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-q}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
K=${2:+-k "$2"}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > $O/gpu_tests.log 2>&1
rc=$?; tail -25 $O/gpu_tests.log | grep -v "^$" | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --knn-ref 0 --sweep-clips 0 > $O/b100k.json 2> $O/b100k.err && \
timeout -k 10 200 python bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --clips 12500 > $O/b12k.json 2> $O/b12k.err
python3 -c "
import json,sys
for f in ['b100k','b12k']:
    try:
        d=json.load(open('$O/'+f+'.json')); r=d['roofline']; print(f, d['ms_per_step'], 'ms', 'frac', r['frac'])
    except Exception as e: print(f, 'ERR', e)
"
