#!/bin/bash
# GPU tests of the current build, its phase stamps at 100k / 12.5k / 1000 clips, and one PMC pass
# (instruction mix) plus one busy-counter pass:  bash tools/r05_st.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05t}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
DO=${DO:-tests stamps pmc}
if [[ $DO == *tests* ]]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -20; exit $rc; }
fi
[[ $DO == *stamps* ]] && for clips in 100000 12500 1000; do
  S=$O/st_$clips; mkdir -p $S
  DSP_ABI_ANY=1 DSP_LIB_PATH=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_stamps.so DIAG_VARIANTS=vad_hamming DIAG_SAVE=$S/s \
    timeout -k 10 200 python tools/diag_extract.py $clips --stamps > $S/diag.log 2>&1 || { tail -20 $S/diag.log; exit 1; }
  echo "== stamps $clips"; python tools/stamps_report.py $S/s_vad_hamming.npy | tee $S/report.txt
  rm -f $S/*.npy  # raw stamps: too large to bring back
done
if [[ $DO == *pmc* ]]; then
bash tools/pmc_insts_var.sh ${T}_pmc base 2>&1 | tee $O/pmc.txt
PMC="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_SALU" \
  bash tools/pmc_insts_var.sh ${T}_busy base 2>&1 | tee $O/pmc_busy.txt
fi
echo R05T_DONE
