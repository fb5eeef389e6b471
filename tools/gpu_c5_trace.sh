#!/bin/bash
# config 5: a per-dispatch kernel trace of two bench steps (the level-synchronous DES's per-level launches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/c5t
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/raw -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 1 --no-cpu > $O/run.log 2>&1 || { echo FAIL; tail $O/run.log; exit 6; }
f=$(find $O/raw -name "*kernel_trace.csv" | head -1)
python3 - $f > $O/levels.txt <<'PY'
import csv,sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'des_' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for r in rows[len(rows)//2:]:
    print(r['Kernel_Name'].split('(')[0][-40:], (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3, 'us grid', r.get('Grid_Size_X', r.get('Grid_Size','')), r.get('Grid_Size_Y',''), r.get('Workgroup_Size_X', ''))
PY
rm -rf $O/raw
cat $O/levels.txt
