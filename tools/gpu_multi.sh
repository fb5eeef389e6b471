#!/bin/bash
# multi-device ABI (libisim RCCL, one rank on the 1-GPU box) + 2-process
# product merge, then the DES tests (plan schedule now topological)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
$T 400 $PT tests/test_multi_gpu.py -m gpu > gpurun_out/multi.log 2>&1 || { tail -40 gpurun_out/multi.log; exit 11; }
tail -1 gpurun_out/multi.log
$T 600 $PT tests/test_des_gpu.py -m gpu > gpurun_out/des.log 2>&1 || { tail -40 gpurun_out/des.log; exit 12; }
tail -1 gpurun_out/des.log
