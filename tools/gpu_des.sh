#!/bin/bash
# DES GPU parity tests (one gpurun call)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_des_gpu.py -m gpu > gpurun_out/des_tests.log 2>&1
rc=$?
tail -40 gpurun_out/des_tests.log
exit $rc
