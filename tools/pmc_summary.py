"""Average rocprofv3 PMC counters per dispatch of a kernel: python tools/pmc_summary.py <dir> [kernel-substr]"""
import collections, csv, glob, os, sys
d = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else "extract_kernel"
split = len(sys.argv) > 3
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if ks in r["Kernel_Name"]:
            agg[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
for k in sorted(agg):
    v = list(agg[k].values())
    print("%-30s n=%3d mean=%.5g" % (k, len(v), sum(v) / len(v)))
