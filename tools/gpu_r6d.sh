#!/bin/bash
# round 6: per-trace change maps in the item engine — its parity suite, the
# c4d bench line and its per-pass trace
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6d
O=gpurun_out/r6d
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_des_items_gpu.py \
  "tests/test_des_gpu.py::test_canonical_with_holds" "tests/test_des_gpu.py::test_cyclic_mode_b_and_wide" > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 600 python bench.py --config c4d > $O/bench_c4d.log 2>&1 || { tail -20 $O/bench_c4d.log; exit 6; }
grep '^{' $O/bench_c4d.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4d', d['value'], d['ms_per_step'], d['config']['des_passes_per_step'], d['config']['des_syncs_per_step'], d['roofline']['frac'])"
bash tools/gpu_c4d_trace.sh 2>&1 | tail -12
