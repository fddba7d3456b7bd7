#!/bin/bash
# VALU/SALU/LDS instruction counts of extract_kernel with phases skipped (diagnostic build):
#   tools/pmc_ablate.sh <tag> mask1 mask2 ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcab_$1; shift
mkdir -p $OUT
export TMPDIR=/tmp DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so
cd /tmp
for m in "$@"; do
  DSP_SKIP=$m timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/m$m -o p -- python3 $R/tools/ablate.py 1000 --once > $OUT/m$m.log 2>&1 || echo "mask $m failed"
done
echo PMC_DONE
