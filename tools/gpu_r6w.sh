#!/bin/bash
# round 6: the c5p line as the driver runs a bench (CPU leg included), twice
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6w
O=gpurun_out/r6w
for r in 1 2; do
timeout -k 10 600 python bench.py --config c5p > $O/bench_c5p_$r.log 2>&1 || { tail -20 $O/bench_c5p_$r.log; exit 6; }
grep '^{' $O/bench_c5p_$r.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c5p', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
