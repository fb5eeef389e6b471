#!/bin/bash
# round 6: wide hot rows without the code-500 table — the wide / site-graph
# parity tests, the c4w and cdag lines, c4w's WRITE_SIZE pass
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6g
O=gpurun_out/r6g
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
  "tests/test_walk_gpu.py::test_tree_wide_forced" "tests/test_walk_gpu.py::test_tree_wide_by_size" \
  "tests/test_walk_gpu.py::test_tree_wide_equals_narrow" "tests/test_walk_gpu.py::test_tree_dag_forced" \
  "tests/test_walk_gpu.py::test_tree_dag_by_size" "tests/test_fullsize_gpu.py::test_config4w_bench_batch" \
  "tests/test_fullsize_gpu.py::test_cdag_bench_batch" "tests/test_des_items_gpu.py::test_items_wide_tree" \
  "tests/test_des_items_gpu.py::test_items_c4w_graph" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for c in c4w cdag; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['roofline']['kernel_ms'], d.get('speedup_vs_wave_walk'), d['cpu_baseline'])"
done
SETS="c4w|--config_c4w" bash tools/gpu_r6_prof.sh
