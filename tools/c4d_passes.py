"""Per-pass summary of an item-engine dispatch trace (tools/gpu_c4d_trace.sh):
the last batch's dispatches split at each k_acc_init (one per pass), with
the pass's GPU-busy time, wall span and dispatch count, and the kernel mix."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last batch: from the last k_gaps (the batch's first kernel)
starts = [i for i, r in enumerate(rows) if "k_gaps" in r["Kernel_Name"]]
rows = rows[starts[-1]:]
passes, cur = [], []
for r in rows:
    if "k_acc_init" in r["Kernel_Name"] and cur:
        passes.append(cur)
        cur = []
    cur.append(r)
passes.append(cur)
tot_busy = tot_span = 0
for n, p in enumerate(passes):
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in p) / 1e6
    span = (int(p[-1]["End_Timestamp"]) - int(p[0]["Start_Timestamp"])) / 1e6
    tot_busy += busy
    tot_span += span
    mix = collections.Counter()
    for r in p:
        mix[r["Kernel_Name"].split("(")[0].split("::")[-1][:24]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    top = ", ".join(f"{k} {v:.2f}" for k, v in mix.most_common(4))
    print(f"pass {n:3d}: {len(p):5d} dispatches, busy {busy:7.2f} ms, span {span:7.2f} ms | {top}")
print(f"total: {sum(len(p) for p in passes)} dispatches, busy {tot_busy:.1f} ms, span {tot_span:.1f} ms")
