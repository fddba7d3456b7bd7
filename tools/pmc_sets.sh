#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over the headline bench for a library variant;
# per-kernel averages into gpurun_out/$TAG/pmc_summary.txt.
#   tools/pmc_sets.sh TAG VARIANT CLIPS   (VARIANT: lib/libdsp_audiorec_<VARIANT>.so, "base" = default)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; V=$2; C=${3:-100000}
O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$V.so; [ "$V" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  DSP_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --no-cfg0 --small-clips 0 --steps 2 --warmup 1 --no-graph --clips $C > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python3 - $O > $O/pmc_summary.txt <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        if "dsp::" not in k: continue
        acc[(k.replace("void ", "")[:32], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("%-32s %-24s n=%3d avg %.6g" % (k, c, len(v), sum(v) / len(v)))
PY
cat $O/pmc_summary.txt
