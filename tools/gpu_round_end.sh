#!/bin/bash
# Round-end evidence in one gpurun call: full GPU suite, smoke, profiles (c3 + c5)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 9; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 8; }
cat gpurun_out/smoke.log
bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { echo PROFILE_FAIL; tail gpurun_out/profile.log; exit 7; }
bash tools/profile_c5.sh > gpurun_out/profile_c5.log 2>&1 || { echo PROFILE_C5_FAIL; tail gpurun_out/profile_c5.log; exit 6; }
bash tools/profile_modeb.sh > gpurun_out/profile_b.log 2>&1 || { echo PROFILE_B_FAIL; tail gpurun_out/profile_b.log; exit 5; }
echo round-end done
