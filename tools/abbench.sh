#!/bin/bash
# A/B on one GPU box with bench.py's own workload (rotating resident batches, graph replay):
#   tools/abbench.sh NAME... [-- extra bench args]; NAME = lib/libdsp_audiorec_NAME.so, "base" = default
# prints per round: name, kernel_avg_ms (HIP events per launch), ms_per_step (graph replay)
R=$(cd "$(dirname "$0")/.." && pwd)
names=(); extra=()
while [ $# -gt 0 ]; do if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi; names+=("$1"); shift; done
for rep in 1 2 3; do
  for v in "${names[@]}"; do
    lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
    out=$(DSP_LIB_PATH=$lib timeout -k 10 120 python3 $R/bench.py --no-cpu "${extra[@]}" 2>/dev/null) || { echo "$v FAILED"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('%-10s kern %.5f ms  step %.5f ms' % ('$v', d['roofline']['kernel_avg_ms'], d['ms_per_step']))"
  done
done
