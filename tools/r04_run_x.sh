#!/bin/bash
# clip-chunk / output-stage size A/B at 100k and 12.5k clips: kernel-trace averages and WRITE_SIZE
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04x}; shift; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp; cd $R
for C in 12500 100000; do
  for v in base "$@"; do
    lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
    (cd /tmp && DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_${v}_$C -o kt -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 10 --clips $C > $O/k_${v}_$C.json 2>&1) || echo "kt $v $C failed"
    (cd /tmp && DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_${v}_$C -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 2 --warmup 1 --no-graph --clips $C > $O/w_${v}_$C.log 2>&1) || echo "pmc $v $C failed"
    k=$(grep -h "extract_kernel<true>" $O/k_${v}_$C/*kernel_stats.csv | cut -d, -f4)
    w=$(python3 $R/tools/pmc_summary.py $O/w_${v}_$C "extract_kernel<true>" | awk '{print $NF}')
    echo "== $C $v kernel_avg_ns $k WRITE_SIZE_KiB $w"
  done
done
rm -rf $O/*/ 2>/dev/null; true
