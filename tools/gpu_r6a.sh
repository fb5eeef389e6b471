#!/bin/bash
# round 6: the new parity tests (c4w bench batch, c4w DES, look-back fault
# path, graph capture, long tie runs, mode-B ancestor marking, the spill ring)
# then the c3 bench line (mode-B legs) and c3p / c4w
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6a
O=gpurun_out/r6a
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  "tests/test_des_items_gpu.py::test_lookback_timeout_fails_loudly" \
  "tests/test_des_items_gpu.py::test_lookback_limit_restored_runs_clean" \
  "tests/test_walk_gpu.py::test_tree_graph_capture" \
  "tests/test_walk_gpu.py::test_tree_spill_two_streams" \
  "tests/test_walk_gpu.py::test_tree_wide_forced" \
  "tests/test_walk_gpu.py::test_reference_topologies" \
  "tests/test_walk_gpu.py::test_mode_b_close_list_depths" \
  "tests/test_kat_gpu.py" "tests/test_golden_records_gpu.py::test_walk_matches_fixture" \
  "tests/test_fullsize_gpu.py::test_mode_b_marking_equals_close_list" \
  "tests/test_fullsize_gpu.py::test_config3_bench_batch_mode_b" \
  "tests/test_fullsize_gpu.py::test_config3p_bench_batch" \
  "tests/test_fullsize_gpu.py::test_config3s_bench_batch" \
  "tests/test_des_items_gpu.py::test_items_match_event_oracle" \
  "tests/test_fullsize_gpu.py::test_config4w_bench_batch" \
  "tests/test_des_items_gpu.py::test_items_c4w_graph" \
  "tests/test_walk_gpu.py::test_tree_dag_forced" "tests/test_walk_gpu.py::test_tree_dag_by_size" \
  "tests/test_fullsize_gpu.py::test_cdag_bench_batch" > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for c in c3 c3p c4w cdag; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['roofline']['kernel_ms'], {k:(d[k]['value'],d[k]['kernel_ms'],d[k]['kernel_kind']) for k in ('mode_b','mode_b_informative') if k in d})"
done
