#!/bin/bash
# kernel-trace stats of one c5 bench run (per-kernel time shares), args: extra bench args
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c5stats; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 3 --warmup 1 --no-cpu "$@" > $O/bench.log 2>&1 || { tail $O/bench.log; exit 11; }
grep "^{" $O/bench.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['value']/1e6,3),'Mtr/s',round(d['roofline']['kernel_ms'],3),'ms',round(d['roofline']['frac'],3))"
f=$(find $O -name '*kernel_stats.csv' | head -1); python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r[:12]: print(x['Name'][:60], x['Calls'], round(float(x['TotalDurationNs'])/1e6,3), 'ms', x['Percentage'][:5])"
