"""Summarise tools/profile_c5.sh output into profiles/<round>/c5 and
profiles/pmc_summary_c5.json (HBM bytes per DES step from PMC).

    python tools/pmc_summary_c5.py gpurun_out/prof_c5 r01

FETCH_SIZE (KiB) is doubled on gfx950 and WRITE_SIZE taken as-is
(/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3); the DES step is the
sum over all des_* dispatches of a step (steps + warmup steps per run).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import occupancy  # noqa: E402


def per_run(path, counter):
    tot = 0.0
    for r in csv.DictReader(open(path)):
        if "des_" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            tot += float(r["Counter_Value"])
    return tot


def main(src, rnd):
    dst = os.path.join(ROOT, "profiles", rnd, "c5")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for p in ("fetch", "write", "sq"):
        if not os.path.exists(os.path.join(src, p, "run_counter_collection.csv")):
            continue
        shutil.copy(os.path.join(src, p, "run_counter_collection.csv"), os.path.join(dst, f"pmc_{p}.csv"))
    line = [l for l in open(os.path.join(src, "stats.log")) if l.startswith("{")][-1]
    open(os.path.join(dst, "bench_under_rocprof.json"), "w").write(line)
    bench = json.loads(line)
    steps = 3  # --steps 2 --warmup 1 in the PMC passes
    fetch = per_run(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE") / steps
    write = per_run(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE") / steps
    stats = list(csv.DictReader(open(os.path.join(src, "stats", "run_kernel_stats.csv"))))
    des_ns = sum(float(r["TotalDurationNs"]) for r in stats if "des_" in r["Name"])
    calls = {r["Name"]: int(r["Calls"]) for r in stats if "des_" in r["Name"]}
    n_steps = bench["steps"] + bench["warmup"]
    out = {
        "round": int(rnd.lstrip("r")), "config": "c5", "batch": bench["config"]["traces_per_rank_per_step"],
        "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --config c5 ; PMC passes --pmc FETCH_SIZE "
                   "| WRITE_SIZE | SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE "
                   "(bench.py --config c5 --steps 2 --warmup 1 --no-cpu)",
        "des_kernel_ns_per_step": des_ns / n_steps,
        "des_calls": calls,
        "fetch_size_kb_per_step": fetch, "write_size_kb_per_step": write,
        "hbm_bytes_per_step": 2 * fetch * 1024 + write * 1024,
        "algorithmic_bytes_per_step": bench["roofline"]["bytes_per_launch"],
        "hbm_bytes_note": "gfx950 correction: FETCH_SIZE doubled; WRITE_SIZE as-is; summed over every des_* "
                          "dispatch of a step",
    }
    sq = os.path.join(src, "sq", "run_counter_collection.csv")
    if os.path.exists(sq):
        # dispatch-time-weighted over every des_* dispatch (pmc_summary.occupancy)
        out["occupancy"] = occupancy(per_run(sq, "SQ_WAVE_CYCLES"), per_run(sq, "GRBM_GUI_ACTIVE"))
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_summary_c5.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
