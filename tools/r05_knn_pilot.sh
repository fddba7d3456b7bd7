#!/bin/bash
# KNN pilot sample sweep (diagnostic library, env DSP_KNN_SAMPLE0 / DSP_KNN_SAMPLE): whole-job time
# at 12.5k and 100k queries for each "s0:s" pair (s0 = 0: no pre-pilot).  bash tools/r05_knn_pilot.sh 0:4096 256:4096 ...
cd ${GRAFT_REPO_ROOT:-.}
export DSP_LIB_PATH=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec_knndiag.so
run() { timeout -k 10 120 python3 tools/bench_knn.py --no-cpu --queries $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['roofline']['frac'], d['fallbacks'])"; }
for rep in 1 2; do
for p in "$@"; do
  s0=${p%%:*}; s=${p##*:}
  echo "s0=$s0 s=$s  12.5k: $(DSP_KNN_SAMPLE0=$s0 DSP_KNN_SAMPLE=$s run 12500)  100k: $(DSP_KNN_SAMPLE0=$s0 DSP_KNN_SAMPLE=$s run 100000)"
done
done
