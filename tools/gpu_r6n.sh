#!/bin/bash
# round 6: the two-kernel fold — kind-7 parity, bench lines, kind-7 profiles
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6n
O=gpurun_out/r6n
timeout -k 10 800 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
  tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_golden_records_gpu.py tests/test_fullsize_gpu.py \
  tests/test_prometheus_gpu.py > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for c in c4 c3p c3s c4w cdag; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['roofline']['kernel_ms'], d.get('speedup_vs_wave_walk'))"
done
SETS="c3p|--config_c3p c3s|--config_c3s c4|--config_c4 c4w|--config_c4w cdag|--config_cdag" bash tools/gpu_r6_prof.sh
