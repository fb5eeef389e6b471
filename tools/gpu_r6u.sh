#!/bin/bash
# round 6: where c5p's time goes (kernel stats of the bench line)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6u
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6u/c5p -o run --output-format csv -- python3 $R/bench.py --config c5p --steps 3 --warmup 1 --no-cpu --no-wave-leg > $R/gpurun_out/r6u/c5p.log 2>&1 || exit 3
python3 - $R/gpurun_out/r6u/c5p <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:80], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms", round(float(r["TotalDurationNs"]) / tot * 100, 1), "%")
PY
