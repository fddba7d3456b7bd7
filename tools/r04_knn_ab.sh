#!/bin/bash
# KNN library A/B with per-kernel times: bench_knn (fallback count) + rocprofv3 kernel stats per
# variant at both shapes.  usage: bash tools/r04_knn_ab.sh TAG variant...  (base = default lib)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  for nq in 12500 100000; do
    echo "== $v $nq $(DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -k 10 200 python3 $R/tools/bench_knn.py --no-cpu --queries $nq | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms"], d["roofline"]["frac"], "fallbacks", d.get("fallbacks"))')"
    (cd /tmp && DSP_ABI_ANY=1 DSP_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$nq -o kt -- python3 $R/tools/bench_knn.py --no-cpu --queries $nq > $O/${v}_$nq.log 2>&1)
    f=$(ls $O/${v}_$nq/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')): print('   %-34s %4s calls avg %8.1f us' % (r['Name'][:34], r['Calls'], float(r['AverageNs'])/1e3))"
  done
done
