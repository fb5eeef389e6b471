#!/bin/bash
# GPU suite on the box: the bench-batch parity tests first (verbose), then the
# whole -m gpu suite, smoke, and the default bench lines named in $BENCH
# (default: c3 c4).  Logs under gpurun_out/suite/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/suite
O=gpurun_out/suite
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py -m gpu -s > $O/fullsize.log 2>&1 || { echo FULLSIZE_FAIL; tail -40 $O/fullsize.log; exit 9; }
grep -E "PASSED|FAILED|max_launch" $O/fullsize.log
if [ -z "$NO_SUITE" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu --deselect tests/test_fullsize_gpu.py > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 $O/gpu_tests.log; exit 8; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 7; }
tail -2 $O/smoke.log
fi
for c in ${BENCH:-c3 c4}; do
timeout -k 10 600 python bench.py --config $c ${BENCH_ARGS} > $O/bench_$c.log 2>&1 || { echo BENCH_${c}_FAIL; tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms frac', round(d['roofline']['frac'],5))"
done
echo suite done
