#!/bin/bash
# instruction-cache counters of extract_kernel per library variant: tools/icache_pmc.sh name...
# (lib/libdsp_audiorec_<name>.so; results in gpurun_out/ic_<name>)
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  DIAG_VARIANTS=vad_hamming DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ --output-format csv -d $R/gpurun_out/ic_$v -o p -- python3 $R/tools/diag_extract.py 1000 > $R/gpurun_out/ic_$v.log 2>&1 || echo "fail $v"
done
