#!/bin/bash
# A/B of extraction-library variants on one box with bench.py's own timing:
#   tools/ab_bench.sh CLIPS name1 name2 ...   (name = lib/libdsp_audiorec_<name>.so, "base" = default lib)
# prints per variant and round: kernel_avg_ms (HIP events) and the roofline fraction.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
clips=$1; shift
for rep in 1 2; do
for v in "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  out=$(DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -k 10 200 python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 10 --clips $clips)
  echo "$v clips=$clips $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("kernel_ms=%s frac=%s step_ms=%s" % (r["kernel_avg_ms"], r["frac"], d["ms_per_step"]))')"
done
done
