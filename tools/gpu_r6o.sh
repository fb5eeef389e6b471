#!/bin/bash
# round 6, after the kind-7 step changes: the whole GPU suite as the driver
# runs it, smoke(), the kind-7 bench lines and their profiles
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6o
O=gpurun_out/r6o
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -2 $O/smoke.log
for c in c4 c3p c3s c4w cdag; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['roofline']['kernel_ms'], d.get('speedup_vs_wave_walk'))"
done
SETS="c3p|--config_c3p c3s|--config_c3s c4|--config_c4 c4w|--config_c4w cdag|--config_cdag" bash tools/gpu_r6_prof.sh
