#!/bin/bash
# Round-4 measurement on the GPU box (no tests): the bench line with rocprofv3 kernel stats and
# FETCH/WRITE PMC at 100k clips (tools/profile_round.sh), the same profile at 12 500 clips (the
# per-rank share at N = 8), the instruction mix and per-phase stamps of the shipping kernel, KNN
# kernel stats at both shapes, and the row-f4 end-to-end breakdown.  usage: bash tools/r04_final.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r04z}
O=$R/gpurun_out/$T; mkdir -p $O; cd $R
export TMPDIR=/tmp
bash tools/profile_round.sh $T
bash tools/profile_round.sh ${T}_12k --clips 12500 --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0
bash tools/pmc_insts_var.sh ${T}_pmc base
bash tools/stamps_seq.sh $T stamps
for nq in 12500 100000; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/knn_kt_$nq -o kt -- python3 $R/tools/bench_knn.py --no-cpu --queries $nq > $O/knn_kt_$nq.log 2>&1)
  timeout -k 10 200 python3 tools/bench_knn.py --queries $nq > $O/knn_$nq.json 2> $O/knn_$nq.err
done
timeout -k 10 300 python3 tools/f4_breakdown.py --files 2000 > $O/f4.json 2> $O/f4.err; cat $O/f4.json
echo FINAL_DONE
