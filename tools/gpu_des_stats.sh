#!/bin/bash
# kernel-trace stats of one DES bench line (2 timed steps), top kernels printed
#   CFG=c4d bash tools/gpu_des_stats.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ds && O=$PWD/gpurun_out/ds
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/st -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-c4d} --steps 2 --warmup 1 --no-cpu > $O/st.log 2>&1 || { tail $O/st.log; exit 4; }
f=$(find $O/st -name 'run_kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us {r['Name'][:80]}")
print('total ms', tot/1e6)
PY
grep '^{' $O/st.log | head -c 300; echo
rm -rf $O/st
