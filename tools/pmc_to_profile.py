"""Fold a profile_round.sh run into profiles/: kernel-trace stats + PMC HBM bytes per launch.

    python tools/pmc_to_profile.py <gpurun_out/TAG> <round-tag> [key]

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; gfx950 FETCH_SIZE counts half
of a wide streaming read -- MI355X_MICROARCH.md, HBM section), averaged over the
extract_kernel dispatches of the PMC passes.  key = "<clips>_<L>_<S>_<window>_<vad>" as bench.py
looks it up; default from the bench.json of the same run.
"""
import collections, csv, glob, json, os, shutil, sys

src, tag = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(d, name, ks="dsp::extract_kernel<"):  # not extract_exact_kernel
    vals = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if ks in r["Kernel_Name"] and r["Counter_Name"] == name:
                vals[(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return sum(vals.values()) / len(vals), len(vals)


bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
cfg = bench["config"]
key = sys.argv[3] if len(sys.argv) > 3 else "%d_%d_%d_%s_%d" % (
    cfg["clips_per_gpu"], cfg["frame_length"], cfg["frame_shift"], cfg["window"], int(cfg["vad"]))
fetch, nf = mean_counter(os.path.join(src, "pmc_fetch"), "FETCH_SIZE")
write, nw = mean_counter(os.path.join(src, "pmc_write"), "WRITE_SIZE")
hbm = int(round((2 * fetch + write) * 1024))
prof = os.path.join(REPO, "profiles")
os.makedirs(prof, exist_ok=True)
pj = os.path.join(prof, "pmc_extract.json")
pm = json.load(open(pj)) if os.path.exists(pj) else {}
pm[key] = {"hbm_bytes_per_launch": hbm, "fetch_size_kib": round(fetch, 2), "write_size_kib": round(write, 2),
           "dispatches": [nf, nw], "source": "profiles/%s_pmc_*.csv (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                             "separate passes; FETCH_SIZE doubled for gfx950)" % tag}
json.dump(pm, open(pj, "w"), indent=1, sort_keys=True)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(prof, "%s_kernel_stats.csv" % tag))
for kind in ("fetch", "write"):
    rows = []
    for f in glob.glob(os.path.join(src, "pmc_" + kind, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "extract_kernel" in r["Kernel_Name"]]
    with open(os.path.join(prof, "%s_pmc_%s.csv" % (tag, kind)), "w", newline="") as o:
        w = csv.writer(o)
        w.writerow(["Dispatch_Id", "Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "Counter_Name", "Counter_Value"])
        for r in rows:
            w.writerow([r["Dispatch_Id"], r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["Counter_Name"], r["Counter_Value"]])
shutil.copy(os.path.join(src, "bench.json"), os.path.join(prof, "%s_bench.json" % tag))
print(key, pm[key])
