"""Summarise a rocprofv3 profile set of bench.py (produced by
tools/profile_cfg.sh) into profiles/pmc_summary_<name>.json and copy the
CSVs judged into profiles/<round>/<name>/.

    python tools/pmc_summary.py gpurun_out/prof_c4 r02 c4

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3): the
FETCH_SIZE and WRITE_SIZE passes run separately; FETCH_SIZE (KiB) is doubled
on gfx950 (it tallies 128-B streaming requests at 64 B), WRITE_SIZE is taken
as-is.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "isim_walk"  # replaced in main() by the profile's dominant isim kernel (isim_walk / isim_tree)


def counters(path):
    agg = collections.defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {"kernel": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                    "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]), "lds": int(r["LDS_Block_Size"]),
                    "scratch": int(r["Scratch_Size"])}
    return {k: sum(v) / len(v) for k, v in agg.items()}, meta


CUS, WAVES_PER_CU = 256, 32  # MI355X: 8 XCDs x 32 CUs; 8 waves/SIMD x 4 SIMDs


def occupancy(wave_cycles, grbm_gui_active, xcds=8):
    """Mean resident waves per CU over the dispatch against the gfx950 limit
    of 32: SQ_WAVE_CYCLES counts quad-cycles summed over every wave
    (MI355X_MICROARCH.md, s_memtime vs SQ PMC units), GRBM_GUI_ACTIVE the
    dispatch's cycles summed over the 8 XCDs (ibid., DVFS give-back)."""
    waves = 4 * wave_cycles / (grbm_gui_active / xcds) / CUS
    return {"mean_waves_per_cu": waves, "peak_waves_per_cu": WAVES_PER_CU, "frac": waves / WAVES_PER_CU,
            "formula": "4*SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE/8) / 256 CUs"}


def main(src, rnd, name):
    dst = os.path.join(ROOT, "profiles", rnd, name)
    os.makedirs(dst, exist_ok=True)
    global KERNEL
    stats_rows = list(csv.DictReader(open(os.path.join(src, "stats", "run_kernel_stats.csv"))))
    # the bench line's own kernel (its launch kind), not other legs' (c3 also times mode B)
    line = json.loads([l for l in open(os.path.join(src, "stats.log")) if l.startswith("{")][-1])
    kind = line["config"]["launch"]["kernel_kind"]
    prefix = "isim::dev::isim_tree<" if kind == 7 else f"isim::dev::isim_walk<{kind},"
    walk = max((r for r in stats_rows if prefix in r["Name"]), key=lambda r: float(r["TotalDurationNs"]))
    KERNEL = walk["Name"].split("(")[0]
    shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "stats", "run_kernel_trace.csv"), os.path.join(dst, "kernel_trace.csv"))
    for p in ("fetch", "write", "sq1", "sq2", "sq3"):
        if os.path.exists(os.path.join(src, p, "run_counter_collection.csv")):
            shutil.copy(os.path.join(src, p, "run_counter_collection.csv"), os.path.join(dst, f"pmc_{p}.csv"))
    bench_line = [l for l in open(os.path.join(src, "stats.log")) if l.startswith("{")][-1]
    with open(os.path.join(dst, "bench_under_rocprof.json"), "w") as f:
        f.write(bench_line)
    bench = json.loads(bench_line)
    fetch, meta = counters(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write, _ = counters(os.path.join(src, "write", "run_counter_collection.csv"))
    sq1, _ = counters(os.path.join(src, "sq1", "run_counter_collection.csv"))
    sq2, _ = counters(os.path.join(src, "sq2", "run_counter_collection.csv"))
    n = bench["config"]["global_batch"] // bench["n_gpus"]
    hops = bench["config"]["hop_visits_per_trace"]
    # per invocation per 64 traces (one wave64's worth of lanes)
    unit = n / 64 * hops
    kernel_ns = float(walk["AverageNs"])
    xcds = 8
    out = {
        "round": int(rnd.lstrip("r")),
        "config": name,
        "batch": n,
        "command": f"tools/profile_cfg.sh {name}: rocprofv3 --kernel-trace --stats -- python3 bench.py "
                   f"{bench_args(src)}; PMC passes: --pmc FETCH_SIZE | WRITE_SIZE | SQ_* (bench.py ... --steps 3 "
                   "--warmup 1 --no-cpu)",
        "kernel": walk["Name"],
        "kernel_avg_ns": kernel_ns,
        "kernel_calls": int(walk["Calls"]),
        "resources": meta,
        "fetch_size_kb_per_launch": fetch["FETCH_SIZE"],
        "write_size_kb_per_launch": write["WRITE_SIZE"],
        "hbm_bytes_per_launch": 2 * fetch["FETCH_SIZE"] * 1024 + write["WRITE_SIZE"] * 1024,
        "hbm_bytes_note": "gfx950 correction: FETCH_SIZE doubled (MI355X_MICROARCH.md §HBM); WRITE_SIZE "
                          "taken as-is (16 B/lane record stores); includes the per-workgroup global-atomic flush",
        "per_invocation_per_64_traces": {
            "valu": sq1["SQ_INSTS_VALU"] / unit, "salu": sq1["SQ_INSTS_SALU"] / unit,
            "smem": sq1["SQ_INSTS_SMEM"] / unit, "lds": sq2["SQ_INSTS_LDS"] / unit},
        "wave_cycle_shares": {
            "wait_any": sq1["SQ_WAIT_ANY"] / sq1["SQ_WAVE_CYCLES"],
            "wait_inst_any": sq1["SQ_WAIT_INST_ANY"] / sq1["SQ_WAVE_CYCLES"],
            "active_inst_any": sq1["SQ_ACTIVE_INST_ANY"] / sq1["SQ_WAVE_CYCLES"]},
        "waves": sq1["SQ_WAVES"],
        "grbm_gui_active": sq2["GRBM_GUI_ACTIVE"],
        "effective_clock_ghz": sq2["GRBM_GUI_ACTIVE"] / xcds / kernel_ns,
        "occupancy": occupancy(sq1["SQ_WAVE_CYCLES"], sq2["GRBM_GUI_ACTIVE"]),
        # a SIMD-32 issues one wave64 VALU instruction per 2 cycles (MI355X_MICROARCH.md, Wave
        # scheduling), so a CU at most 2 per cycle; multi-pass instructions (v_mad_u64_u32 of the
        # Philox rounds) hold the SIMD longer, so a VALU-bound kernel can sit well below 1 here
        "valu_issue_frac": sq1["SQ_INSTS_VALU"] / (2 * sq2["GRBM_GUI_ACTIVE"] / xcds * CUS),
        "valu_issue_formula": "SQ_INSTS_VALU / (2 per CU-cycle x GRBM_GUI_ACTIVE/8 x 256 CUs)",
        "salu_issue_frac": sq1["SQ_INSTS_SALU"] / (sq2["GRBM_GUI_ACTIVE"] / xcds * CUS),
    }
    sq3_path = os.path.join(src, "sq3", "run_counter_collection.csv")
    if os.path.exists(sq3_path):
        sq3, _ = counters(sq3_path)
        if sq3.get("SQ_ACTIVE_INST_VALU"):
            # lanes doing work per VALU instruction (SQ_THREAD_CYCLES_VALU counts
            # thread-cycles, SQ_ACTIVE_INST_VALU instruction-cycles; x64 lanes)
            out["valu_lane_utilisation"] = sq3["SQ_THREAD_CYCLES_VALU"] / (64.0 * sq3["SQ_ACTIVE_INST_VALU"])
        out["sq3"] = sq3
    with open(os.path.join(ROOT, "profiles", f"pmc_summary_{name}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def bench_args(src):
    return open(os.path.join(src, "args")).read().strip() if os.path.exists(os.path.join(src, "args")) else ""


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
