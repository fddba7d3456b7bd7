#!/bin/bash
# dynamic instruction counts of extract_kernel per library variant: tools/pmc_insts.sh name...
# (lib/libdsp_audiorec_<name>.so; results in gpurun_out/pi_<name>)
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  DIAG_VARIANTS=vad_hamming DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/pi_$v -o p -- python3 $R/tools/diag_extract.py 1000 > $R/gpurun_out/pi_$v.log 2>&1 || echo "fail $v"
  DIAG_VARIANTS=vad_hamming DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d $R/gpurun_out/pi2_$v -o p -- python3 $R/tools/diag_extract.py 1000 > $R/gpurun_out/pi2_$v.log 2>&1 || echo "fail $v"
done
