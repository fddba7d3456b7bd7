#!/bin/bash
# One PMC pass (instruction mix + wave states, or the counters in $PMC) per library variant at 100k clips, summarised:
#   bash tools/pmc_insts_var.sh TAG variant...   (variant: lib/libdsp_audiorec_<v>.so, base = default)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift
O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  (cd /tmp && DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY} \
     --output-format csv -d $O/$v -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 2 --warmup 1 --no-graph --clips 100000 > $O/$v.log 2>&1) || { echo "pmc $v failed"; tail -3 $O/$v.log; }
  echo "== $v"; python3 $R/tools/pmc_summary.py $O/$v "extract_kernel<true>"| sed 's/^/  /'
done
