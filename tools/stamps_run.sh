#!/bin/bash
# Per-phase stamps of the extraction kernel at CLIPS clips (diagnostic build, libdsp_audiorec_stamps.so):
#   tools/stamps_run.sh TAG [CLIPS]  -> gpurun_out/st_TAG/report.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; C=${2:-100000}; O=$R/gpurun_out/st_$T; mkdir -p $O; cd $R
DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so DIAG_VARIANTS=vad_hamming DIAG_SAVE=$O/s \
  timeout -k 10 200 python tools/diag_extract.py $C --stamps > $O/diag.log 2>&1 || { tail -20 $O/diag.log; exit 1; }
python tools/stamps_pipe.py $O/s_vad_hamming.npy > $O/report.txt 2>&1; cat $O/report.txt
