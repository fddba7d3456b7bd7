#!/bin/bash
# kernel durations (rocprofv3 --kernel-trace --stats) of the headline bench per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  (cd /tmp && DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o kt -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 10 > $O/$v.json 2> $O/$v.err) || { echo "kt $v failed"; tail -3 $O/$v.err; }
  echo "== $v $(python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["roofline"]["kernel_avg_ms"], d["ms_per_step"])' $O/$v.json)"
  f=$(ls $O/$v/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && grep -E "extract" $f | cut -c1-160
done
