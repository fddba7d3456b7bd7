#!/bin/bash
# PMC passes over tools/bench_knn.py (one counter set per run): tools/pmc_knn.sh TAG QUERIES [env assignments]
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; Q=$2; shift 2
O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  env "$@" timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o p -- python3 $R/tools/bench_knn.py --no-cpu --queries $Q > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        if "screen" not in k: continue
        acc[(k.replace("void ", "")[:30], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("%-30s %-26s n=%3d avg %.6g" % (k, c, len(v), sum(v) / len(v)))
PY
