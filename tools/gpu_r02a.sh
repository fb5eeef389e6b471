#!/bin/bash
# round 2: the new GPU tests (KATs on every kernel kind, informative mode B,
# u32 counter guard, config-5 at bench scale), then the full -m gpu suite,
# then bench lines (default c3 with the mode-B legs, c1).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
$T 600 $PT tests/test_kat_gpu.py \
  "tests/test_walk_gpu.py::test_config3_mode_b_informative" "tests/test_walk_gpu.py::test_site_counter_beyond_u32" \
  "tests/test_des_gpu.py::test_config5_bench_scale" -m gpu > gpurun_out/new.log 2>&1 || { tail -40 gpurun_out/new.log; exit 11; }
tail -1 gpurun_out/new.log
$T 900 $PT tests -m gpu > gpurun_out/all.log 2>&1 || { tail -40 gpurun_out/all.log; exit 12; }
tail -1 gpurun_out/all.log
$T 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b_c3.log 2>&1 || { tail -5 gpurun_out/b_c3.log; exit 13; }
tail -1 gpurun_out/b_c3.log
$T 300 python bench.py --config c1 --steps 10 --warmup 3 > gpurun_out/b_c1.log 2>&1 || { tail -5 gpurun_out/b_c1.log; exit 14; }
tail -1 gpurun_out/b_c1.log
