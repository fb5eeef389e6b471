"""Summarise tools/profile_des.sh output into profiles/<round>/<name> and
profiles/pmc_summary_<name>.json: HBM bytes per DES step from PMC, and the
dispatch-time-weighted mean resident waves per CU.

    python tools/pmc_summary_des.py gpurun_out/prof_c4d r05 c4d

FETCH_SIZE (KiB) is doubled on gfx950 and WRITE_SIZE taken as-is
(/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3).  A step is every
dispatch of one DES batch: the des_* kernels of the level-synchronous engine
(c5), or — the item engine (c5p, c4d) — all of its dispatches (its k_* kernels,
the rocPRIM sorts and scans, the runtime's fills and copies).  The PMC passes
run two batches (--steps 1 --warmup 1).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# where profiles/ is written (ISIM_PROF_OUT: e.g. gpurun_out/ on the GPU box, copied back from there)
OUT = os.environ.get("ISIM_PROF_OUT", os.path.join(ROOT, "profiles"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import occupancy  # noqa: E402


def mine(name, kernel):
    return "des_" in kernel if name == "c5" else True


def per_run(path, counter, name):
    tot = 0.0
    for r in csv.DictReader(open(path)):
        if mine(name, r["Kernel_Name"]) and r["Counter_Name"] == counter:
            tot += float(r["Counter_Value"])
    return tot


def per_kernel(paths, name):
    """Counter sums per kernel name over the PMC passes (the raw per-dispatch
    files of an item-engine step run to tens of MB)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in paths:
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            if mine(name, r["Kernel_Name"]):
                agg[r["Kernel_Name"].split("(")[0][:120]][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main(src, rnd, name):
    dst = os.path.join(OUT, rnd, name)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    agg = per_kernel([os.path.join(src, p, "run_counter_collection.csv") for p in ("fetch", "write", "sq")], name)
    names = sorted({c for v in agg.values() for c in v})
    with open(os.path.join(dst, "pmc_per_kernel.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel"] + names)
        for k in sorted(agg, key=lambda k: -agg[k].get("FETCH_SIZE", 0.0)):
            w.writerow([k] + [agg[k].get(c, 0.0) for c in names])
    line = [l for l in open(os.path.join(src, "stats.log")) if l.startswith("{")][-1]
    open(os.path.join(dst, "bench_under_rocprof.json"), "w").write(line)
    bench = json.loads(line)
    steps = 2  # --steps 1 --warmup 1 in the PMC passes
    fetch = per_run(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE", name) / steps
    write = per_run(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE", name) / steps
    stats = list(csv.DictReader(open(os.path.join(src, "stats", "run_kernel_stats.csv"))))
    n_steps = bench["steps"] + bench["warmup"]
    ns = sum(float(r["TotalDurationNs"]) for r in stats if mine(name, r["Name"]))
    calls = sum(int(r["Calls"]) for r in stats if mine(name, r["Name"]))
    out = {
        "round": int(rnd.lstrip("r")), "config": name, "batch": bench["config"]["traces_per_rank_per_step"],
        "command": f"tools/profile_des.sh {name}: rocprofv3 --kernel-trace --stats -- python3 bench.py --config "
                   f"{name}; PMC passes --pmc FETCH_SIZE | WRITE_SIZE | SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES "
                   f"GRBM_GUI_ACTIVE (bench.py --config {name} --steps 1 --warmup 1 --no-cpu)",
        "kernel_ns_per_step": ns / n_steps,
        "dispatches_per_step": calls / n_steps,
        "fetch_size_kb_per_step": fetch, "write_size_kb_per_step": write,
        "hbm_bytes_per_step": 2 * fetch * 1024 + write * 1024,
        "algorithmic_bytes_per_step": bench["roofline"]["bytes_per_launch"],
        "hbm_bytes_note": "gfx950 correction: FETCH_SIZE doubled; WRITE_SIZE as-is; summed over every dispatch of "
                          "a step" + (" (des_* kernels)" if name == "c5" else " (the item engine's kernels, rocPRIM "
                                                                              "sorts/scans, fills, copies)"),
    }
    out["hbm_over_algorithmic"] = out["hbm_bytes_per_step"] / max(1, out["algorithmic_bytes_per_step"])
    sq = os.path.join(src, "sq", "run_counter_collection.csv")
    if os.path.exists(sq):
        out["occupancy"] = occupancy(per_run(sq, "SQ_WAVE_CYCLES", name), per_run(sq, "GRBM_GUI_ACTIVE", name))
    json.dump(out, open(os.path.join(OUT, f"pmc_summary_{name}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
