#!/bin/bash
# bench_knn per library variant (lib/libdsp_audiorec_NAME.so; "base" = default), shard and full
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  for nq in 12500 100000; do
    echo -n "$v $nq: "
    DSP_LIB_PATH=$lib timeout -k 10 200 python3 $R/tools/bench_knn.py --no-cpu --queries $nq | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms'], d['roofline']['frac'])"
  done
done
