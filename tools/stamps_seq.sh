#!/bin/bash
# Per-phase stamps of the one-clip-per-workgroup extraction kernel for stamp-build variants:
#   tools/stamps_seq.sh TAG variant...  (variant: lib/libdsp_audiorec_<v>.so; "stamps" = current)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; cd $R
for v in "$@"; do
  O=$R/gpurun_out/st_${T}_$v; mkdir -p $O
  DSP_ABI_ANY=1 DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so DIAG_VARIANTS=vad_hamming DIAG_SAVE=$O/s \
    timeout -k 10 200 python tools/diag_extract.py 100000 --stamps > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
  echo "== $v"; python tools/stamps_report.py $O/s_vad_hamming.npy | tee $O/report.txt
done
