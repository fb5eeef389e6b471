#!/bin/bash
# DES parity, then A/B of libisim_base.so vs libisim.so on config 5
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_des_gpu.py -m gpu > gpurun_out/des.log 2>&1 || { tail -30 gpurun_out/des.log; exit 12; }
[ -n "$NOTEST" ] || tail -1 gpurun_out/des.log
REPS=2 LIBS="${LIBS:-libisim_base.so libisim.so}" CONFIGS="--config c5" bash tools/ab_libs.sh
