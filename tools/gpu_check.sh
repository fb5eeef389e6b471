set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 9; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 8; }
tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench_default.log; exit 7; }
tail -1 gpurun_out/bench_default.log
