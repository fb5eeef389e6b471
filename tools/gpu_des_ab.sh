set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_des_gpu.py tests/test_golden_records_gpu.py -m gpu > gpurun_out/des_tests.log 2>&1 || { tail -30 gpurun_out/des_tests.log; exit 12; }
tail -1 gpurun_out/des_tests.log
LIBS="libisim_base.so libisim.so" bash tools/gpu_ab_c5.sh
