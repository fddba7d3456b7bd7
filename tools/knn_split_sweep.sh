#!/bin/bash
# KNN reference-split sweep on the GPU box: bench_knn at the given query count for each forced
# split count (DSP_KNN_NSPLIT) and the model's own pick.  usage: tools/knn_split_sweep.sh Q s1 s2 ...
# Needs the diagnostic library (make -C dsp-audioreclabs_amd/csrc knndiag): the product library
# reads no environment variables.
cd ${GRAFT_REPO_ROOT:-.}
export DSP_LIB_PATH=$PWD/dsp-audioreclabs_amd/lib/libdsp_audiorec_knndiag.so
Q=$1; shift
run() { timeout -k 10 120 python3 tools/bench_knn.py --no-cpu --queries $Q | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['roofline']['frac'])"; }
echo "Q=$Q model: $(run)"
for s in "$@"; do echo "Q=$Q nsplit=$s: $(DSP_KNN_NSPLIT=$s run)"; done
