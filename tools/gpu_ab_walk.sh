#!/bin/bash
# walk parity tests, then an A/B of libisim_base.so vs libisim.so on the given bench configs
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_walk_gpu.py tests/test_fullsize_gpu.py -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 12; }
tail -1 gpurun_out/t.log
REPS=2 LIBS="libisim_base.so libisim.so" CONFIGS="${1:---config c4}" bash tools/ab_libs.sh
