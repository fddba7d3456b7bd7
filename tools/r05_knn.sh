#!/bin/bash
# Round 5 KNN check: bench_knn at both shapes (whole job) for each library variant, and the
# kernel-trace stats of the current build at both shapes (pilot and main screen as separate kernels)
#   bash tools/r05_knn.sh TAG [variant...]   (variant: lib/libdsp_audiorec_<v>.so; base = current)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r05k}; shift; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
for rep in 1 2; do
for v in "$@" base; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  for nq in 12500 100000; do
    echo "$v nq=$nq $(DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -k 10 200 python3 tools/bench_knn.py --no-cpu --queries $nq)" | tee -a $O/knn_ab.txt
  done
done
done
for nq in 12500 100000; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$nq -o kt -- python3 $R/tools/bench_knn.py --no-cpu --queries $nq > $O/kt_$nq.log 2>&1) || exit 1
done
find $O -name "*kernel_stats.csv" | head
echo R05K_DONE
