#!/bin/bash
# PMC comparison of the extraction kernels on bench's workload (separate passes per counter set)
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for k in hop generic; do
  if [ $k = generic ]; then export DSP_EXTRACT_KERNEL=generic; else unset DSP_EXTRACT_KERNEL; fi
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pc_${k}_$i -o p -- python3 $R/bench.py --no-cpu --steps 5 --warmup 1 > $R/gpurun_out/pc_${k}_$i.log 2>&1 || { echo "fail $k $i"; exit 1; }
  done
done
for i in 1 2 3; do python3 $R/tools/pmc_summary.py $R/gpurun_out/pc_hop_$i hop_kernel; done > $R/gpurun_out/pc_hop.txt 2>&1
for i in 1 2 3; do python3 $R/tools/pmc_summary.py $R/gpurun_out/pc_generic_$i extract_kernel; done > $R/gpurun_out/pc_generic.txt 2>&1
echo done
