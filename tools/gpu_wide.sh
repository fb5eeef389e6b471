#!/bin/bash
# Wide lane-tree walks: the c4w line (a 100k-service realistic graph at
# probability 30: 100,000 positions) with its wave-interpreter leg and CPU
# baseline, then c3p under ISIM_TREE_FORCE_WIDE against the 8-byte nodes
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide
O=gpurun_out/wide
timeout -k 10 600 python -u bench.py --config c4w --steps 5 --warmup 2 > $O/c4w.log 2>&1 || { tail -20 $O/c4w.log; exit 1; }
grep '^{' $O/c4w.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print("c4w", round(d["value"]/1e6,2), "M/s", round(d["ms_per_step"],2), "ms", d["config"]["launch"], "wave", round(d["wave_walk"]["value"]/1e6,3), "x", round(d["speedup_vs_wave_walk"],1), "cpu", round(d["cpu_baseline"]["value"]))'
for v in "" 1 "" 1; do
  env ${v:+ISIM_TREE_FORCE_WIDE=1} timeout -k 10 300 python -u bench.py --config c3p --steps 5 --warmup 2 --no-cpu --no-wave-leg > $O/c3p.log 2>&1 || { tail -20 $O/c3p.log; exit 1; }
  echo "c3p wide=${v:-0} $(grep '^{' $O/c3p.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,2), "M/s", round(d["ms_per_step"],2), "ms")')"
done
