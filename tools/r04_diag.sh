#!/bin/bash
# Stamps of a variant library and PMC instruction/wave-state counters of variants (A/B diagnosis).
#   bash tools/r04_diag.sh TAG STAMPS_VARIANT PMC_VARIANT...
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; SV=$2; shift 2
O=$R/gpurun_out/$T; mkdir -p $O; cd $R
DSP_ABI_ANY=1 DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$SV.so DIAG_VARIANTS=vad_hamming DIAG_SAVE=$O/s \
  timeout -k 10 200 python tools/diag_extract.py 100000 --stamps > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
python tools/stamps_pipe.py $O/s_vad_hamming.npy | tee $O/report_$SV.txt
for v in "$@"; do
  DSP_ABI_ANY=1 bash tools/pmc_sets.sh ${T}_pmc_$v $v 100000 > /dev/null 2>&1 || true
  echo "== $v"; cat $R/gpurun_out/${T}_pmc_$v/pmc_summary.txt
done
echo DIAG_DONE
