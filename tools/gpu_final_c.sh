#!/bin/bash
# full GPU suite, then the c3 profile set (stats + PMC) and mode-B stats
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/final/gpu_tests.log; exit 9; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 8; }
timeout -k 10 600 python bench.py > gpurun_out/final/bench_c3.log 2>&1 || { echo BENCH_FAIL; exit 7; }
bash tools/profile_cfg.sh c3 "--config c3 --no-mode-b" > gpurun_out/prof_c3.log 2>&1 || { echo PROF_C3_FAIL; tail gpurun_out/prof_c3.log; exit 6; }
bash tools/profile_modeb.sh > gpurun_out/prof_b.log 2>&1 || { echo PROF_B_FAIL; exit 5; }
echo final C done
