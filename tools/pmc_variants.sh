#!/bin/bash
# SQ_INSTS_VALU / SALU / LDS and kernel time per library variant (hop kernel), bench workload
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  export DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/pv_$v -o p -- python3 $R/bench.py --no-cpu --steps 5 --warmup 1 > $R/gpurun_out/pv_$v.log 2>&1 || { echo "fail $v"; continue; }
  echo "== $v"; python3 $R/tools/pmc_summary.py $R/gpurun_out/pv_$v hop_kernel
done
