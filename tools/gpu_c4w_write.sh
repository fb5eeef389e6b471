#!/bin/bash
# c4w WRITE_SIZE per launch under settings: default, no duration rows
# (--no-svc-dur), no records (--no-records) — where the wide kernel's writes go
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c4ww
mkdir -p $O
for v in "" "--no-svc-dur" "--no-records" "--no-svc-dur --no-records"; do
  tag=$(echo "x$v" | tr -d ' -')
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/$tag -o run --output-format csv -- python3 $R/bench.py --config c4w --steps 2 --warmup 1 --no-cpu --no-wave-leg $v > $O/$tag.log 2>&1 || { echo FAIL $tag; tail -5 $O/$tag.log; exit 1; }
  python3 - $O/$tag <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = {}; n = {}
for r in csv.DictReader(open(f)):
    if "isim_tree" not in r["Kernel_Name"]: continue
    k = r["Dispatch_Id"]
    tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
v = sorted(tot.values())
print(sys.argv[1].split("/")[-1], "launches", len(v), "WRITE_SIZE KB per launch (median)", v[len(v)//2])
PY
done
