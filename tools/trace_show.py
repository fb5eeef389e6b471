"""Summarise a per-dispatch kernel trace of DES steps (tools/trace_c5.sh):
the last step's des_* dispatches in launch order with grid and duration."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "des_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "des_arrivals" in r["Kernel_Name"]]
step = rows[starts[-1]:]
tot = 0
by = {}
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    by.setdefault(k, [0, 0.0])
    by[k][0] += 1
    by[k][1] += d
    if len(sys.argv) > 2:
        print(f"{k:22s} grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):7d} x {r['Workgroup_Size_X']:5s} {d:9.1f} us")
span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
print(f"step: {len(step)} dispatches, busy {tot:.0f} us, span {span:.0f} us")
for k, (n, d) in sorted(by.items(), key=lambda x: -x[1][1]):
    print(f"  {k:22s} {n:5d} {d:9.0f} us")
