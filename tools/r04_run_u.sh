#!/bin/bash
# clip-queue chunk A/B: kernel-trace durations and WRITE_SIZE per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04u}; shift; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp; cd $R
bash tools/r04_kt.sh $T base "$@"
for v in base "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  (cd /tmp && DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$v -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 2 --warmup 1 --no-graph > $O/w_$v.log 2>&1) || echo "pmc $v failed"
  echo "== $v WRITE_SIZE"; python3 $R/tools/pmc_summary.py $O/w_$v "extract_kernel<true>"
done
rm -rf $O/*/ 2>/dev/null; true
