#!/bin/bash
# instruction mix (one PMC pass per variant) and phase ablation timings at 100k clips:
#   bash tools/r05_pmc.sh TAG "pmc variants" "ablation variants"
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
bash tools/pmc_insts_var.sh $T $2 2>&1 | tee $O/pmc.txt
[ -n "$3" ] && timeout -k 10 600 bash tools/ab_bench.sh 100000 $3 2>&1 | grep -v amdgpu.ids | tee $O/abl.txt
echo R05P_DONE
