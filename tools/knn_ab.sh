#!/bin/bash
# KNN A/B on the GPU box: parity tests, then bench_knn per screen variant / split target
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gtk.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/gtk.log
run() { timeout -k 10 200 python3 tools/bench_knn.py --no-cpu "$@" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['queries'], d['ms'], d['roofline']['frac'])"; }
for scr in s t; do for t in ${TARGETS:-512 2048}; do
  echo -n "screen=$scr wgs=$t shard: "; DSP_KNN_SCREEN=$scr DSP_KNN_TARGET_WGS=$t run
  echo -n "screen=$scr wgs=$t full:  "; DSP_KNN_SCREEN=$scr DSP_KNN_TARGET_WGS=$t run --queries 100000
done; done
