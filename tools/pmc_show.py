"""Print per-launch averages of the walk kernel's counters from tools/pmc_quick.sh output."""
import collections, csv, glob, os, sys
base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcq"
for d in sorted(glob.glob(os.path.join(base, "p[0-9]*/"))):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "isim_walk" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    args = open(d.rstrip("/") + ".args").read().strip() if os.path.exists(d.rstrip("/") + ".args") else d
    print(args, {k: f"{sum(v) / len(v):.4g}" for k, v in sorted(agg.items())})
