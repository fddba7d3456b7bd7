#!/bin/bash
# instruction mix of base and phase ablations, then VALU/SALU/LDS busy counters of base:
#   bash tools/r05_pmc2.sh TAG "variants"
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
bash tools/pmc_insts_var.sh $T $2 2>&1 | tee $O/pmc.txt
PMC="SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_CYCLES_SALU" \
  bash tools/pmc_insts_var.sh ${T}_busy base 2>&1 | tee $O/pmc_busy.txt
echo R05P2_DONE
