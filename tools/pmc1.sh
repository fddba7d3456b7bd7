#!/bin/bash
# One PMC pass (instruction mix) of bench.py's 100k-clip extraction for a library variant:
#   tools/pmc1.sh NAME  (lib/libdsp_audiorec_NAME.so, "base" = default)  -> per-clip counts
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp; cd /tmp; O=$R/gpurun_out/pmc_$1; mkdir -p $O
lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$1.so; [ "$1" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
DSP_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $O/p -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --steps 2 --warmup 1 --no-graph > $O/p.log 2>&1
python3 - $O $1 <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "extract_kernel" not in r.get("Kernel_Name", ""): continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], " ".join("%s=%.0f" % (c.replace("SQ_", ""), sum(v) / len(v) / 100000) for c, v in sorted(acc.items())))
PY
rm -rf $O/p
