#!/bin/bash
# dynamic instruction counts with each phase doubled (diagnostic build): tools/pmc_double.sh tag
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcdbl_$1
mkdir -p $OUT
export TMPDIR=/tmp DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so
cd /tmp
for m in ${MASKS:-0 256 512 1024 2048 4096 8192 16384 32768}; do
  DSP_SKIP=$m timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $OUT/m$m -o p -- python3 $R/tools/ablate.py 1000 --once > $OUT/m$m.log 2>&1 || echo "mask $m failed"
done
echo PMC_DONE
