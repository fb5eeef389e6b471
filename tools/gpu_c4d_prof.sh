#!/bin/bash
# c4d: bench line without debug output, then one kernel-trace --stats profile (per-kernel split of a step)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c4dp
O=$GRAFT_REPO_ROOT/gpurun_out/c4dp
for v in "" "ISIM_DES_ITEMS_NO_INCR=1"; do
  timeout -k 10 400 env $v python bench.py --config c4d --no-cpu --steps 3 --warmup 1 > $O/c4d_$v.log 2>&1 || { echo C4D_FAIL $v; tail $O/c4d_$v.log; exit 7; }
  grep '^{' $O/c4d_$v.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4d [$v]', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],1),'ms')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c4d --no-cpu --steps 1 --warmup 1 > $O/prof.log 2>&1 || { echo PROF_FAIL; tail $O/prof.log; exit 6; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 - $O/kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.1f} ms {int(r['Calls']):7d} calls {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:90]}")
print('total', tot/1e6, 'ms')
PY
echo done
