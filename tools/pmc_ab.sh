#!/bin/bash
# first PMC pass (instruction counts, wave cycles) + timing for library variants:
#   tools/pmc_ab.sh TAG name1 name2 ...  (lib/libdsp_audiorec_<name>.so, "base" = default)
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift
O=$R/gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
for v in "$@"; do
  lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec_$v.so; [ "$v" = base ] && lib=$R/dsp-audioreclabs_amd/lib/libdsp_audiorec.so
  DSP_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT} --output-format csv -d $O/$v -o p -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --steps 4 --warmup 1 --clips 12500 > $O/$v.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.log; exit 1; }
  python3 - $O/$v <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        if "dsp::" not in k: continue
        acc[(k.replace("void ", "")[:28], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("  %-28s %-22s per clip %10.1f" % (k, c, sum(v) / len(v) / 12500))
PY
  DSP_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_kt -o kt -- python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --steps 10 > $O/${v}_kt.log 2>&1 || { echo "$v kt failed"; exit 1; }
  python3 - $O/${v}_kt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "dsp::" in r["Name"]:
        print("  %-44s calls %4s avg_us %9.1f" % (r["Name"].replace("void ", "")[:44], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  out=$(DSP_LIB_PATH=$lib timeout -k 10 200 python3 $R/bench.py --no-cpu --knn-ref 0 --sweep-clips 0 --steps 10)
  echo "$v $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("kernel_ms(100k) %s frac %s" % (d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"]))')"
done
