"""Summarise tools/pmc_des.sh: per des_* kernel (last step), VALU / SALU
issue fractions (wave instructions / (cycles x 256 CUs)) and occupancy."""
import collections
import csv
import glob
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_des"


def rows(p):
    f = glob.glob(os.path.join(base, p, "**", "*counter_collection.csv"), recursive=True)[0]
    out = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "des_" in r["Kernel_Name"]:
            out[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            out[int(r["Dispatch_Id"])]["name"] = r["Kernel_Name"].split("(")[0].split("::")[-1]
    return out


a, b = rows("p1"), rows("p2")
ids_a, ids_b = sorted(a), sorted(b)
n = min(len(ids_a), len(ids_b))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for ia, ib in zip(ids_a[-n // 2:], ids_b[-n // 2:]):  # the timed step (second half)
    ra, rb = a[ia], b[ib]
    k = ra["name"]
    for c, v in ra.items():
        if c != "name":
            agg[k][c] += v
    agg[k]["GRBM_GUI_ACTIVE"] += rb.get("GRBM_GUI_ACTIVE", 0)
for k, d in sorted(agg.items(), key=lambda x: -x[1]["GRBM_GUI_ACTIVE"]):
    cyc = d["GRBM_GUI_ACTIVE"] / 8
    if cyc <= 0:
        continue
    print(f"{k:40s} cycles {cyc:11.0f}  valu {d['SQ_INSTS_VALU'] / cyc / 256:5.2f}  salu {d['SQ_INSTS_SALU'] / cyc / 256:5.2f}"
          f"  lds {d['SQ_INSTS_LDS'] / cyc / 256:5.2f}  waves/CU {4 * d['SQ_WAVE_CYCLES'] / cyc / 256:5.1f}"
          f"  vmem_rd {d['SQ_INSTS_VMEM_RD'] / cyc / 256:5.3f}")
