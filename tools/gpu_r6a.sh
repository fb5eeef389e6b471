#!/bin/bash
# round 6: the new parity tests (c4w bench batch, c4w DES, look-back fault
# path, graph capture, long tie runs) then the spill / DES item suites
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6a
O=gpurun_out/r6a
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  "tests/test_des_items_gpu.py::test_lookback_timeout_fails_loudly" \
  "tests/test_des_items_gpu.py::test_lookback_limit_restored_runs_clean" \
  "tests/test_walk_gpu.py::test_tree_graph_capture" \
  "tests/test_walk_gpu.py::test_tree_spill_two_streams" \
  "tests/test_des_items_gpu.py::test_items_match_event_oracle" \
  "tests/test_fullsize_gpu.py::test_config4w_bench_batch" \
  "tests/test_des_items_gpu.py::test_items_c4w_graph" > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40
exit $rc
