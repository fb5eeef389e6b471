#!/bin/bash
# Round-end evidence, part A: full GPU suite, smoke, bench lines (c3 default,
# c1, c4, c3p, c3s, c4w, c5p, c4d, c5; the item-engine lines before config 5, whose
# ~170 GB the driver may still hold afterwards)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
O=gpurun_out/final
if [ -z "$NO_SUITE" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 $O/gpu_tests.log; exit 9; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 8; }
fi
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_c3.log; exit 7; }
for c in ${BENCH:-c1 c4 c3p c3s c4w c5p c4d c5}; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { echo BENCH_${c}_FAIL; tail -20 $O/bench_$c.log; exit 6; }
done
for c in c3 ${BENCH:-c1 c4 c3p c3s c4w c5p c4d c5}; do grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms frac', round(d['roofline']['frac'],5), 'traffic', d['roofline'].get('traffic'))"; done
echo final A done
