#!/bin/bash
# rocprofv3 PMC passes (one counter set per run) over the bench at 12 500 clips; per-kernel
# averages of each counter into gpurun_out/$1/pmc_summary.txt.  usage: tools/pmc_pass.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-pmc}; shift || true
O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --steps 4 --warmup 1 --clips 12500 "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - $O > $O/pmc_summary.txt <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
        if "dsp::" not in k: continue
        acc[(k.replace("void ", "")[:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("%-40s %-24s n=%3d avg %.6g" % (k, c, len(v), sum(v) / len(v)))
PY
cat $O/pmc_summary.txt
