#!/bin/bash
# round 6: k_tiefix's move budget — the item-engine parity suite, c5p / c4d lines
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6t
O=gpurun_out/r6t
timeout -k 10 800 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
  tests/test_des_items_gpu.py > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for c in c5p c4d; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['ms_per_step'], d['config'].get('des_passes_per_step'), d['config'].get('des_syncs_per_step'))"
done
