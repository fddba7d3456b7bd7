#!/bin/bash
# Phase stamps of a stamps-built library variant at CLIPS clips:
#   tools/stamps_var.sh TAG LIBNAME [CLIPS]   (lib/libdsp_audiorec_<LIBNAME>.so built with -DDSP_STAMPS)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; V=$2; C=${3:-100000}; O=$R/gpurun_out/st_$T; mkdir -p $O; cd $R
DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$V.so DIAG_VARIANTS=vad_hamming DIAG_SAVE=$O/s \
  timeout -k 10 200 python tools/diag_extract.py $C --stamps > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
python tools/stamps_report.py $O/s_vad_hamming.npy > $O/report.txt 2>&1; cat $O/report.txt
