#!/bin/bash
# round 6: the close reads its call site only on a 500 — timing A/B against
# the previous build (libisim_prev.so), with scan budgets 2 and 4 (TW_SCAN),
# then the kind-7 parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6l
O=gpurun_out/r6l
for c in c3p c3s c4w c4; do
  echo "== $c"
  LIBS="libisim_prev.so libisim.so libisim_s2.so libisim_s4.so" CFG="--config $c" REPS=2 timeout -k 10 400 bash tools/gpu_ab.sh || exit 7
done
timeout -k 10 800 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
  tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_golden_records_gpu.py \
  "tests/test_fullsize_gpu.py::test_config3p_bench_batch" "tests/test_fullsize_gpu.py::test_config3s_bench_batch" \
  "tests/test_fullsize_gpu.py::test_config4w_bench_batch" "tests/test_fullsize_gpu.py::test_config4_bench_batch" > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
