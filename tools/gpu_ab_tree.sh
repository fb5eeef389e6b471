#!/bin/bash
# kind-7 parity (tree kernels) then A/B of libisim variants on config 4
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_walk_gpu.py -m gpu -k "mesh or probability or tree or refill" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 12; }
[ -n "$NOTEST" ] || tail -1 gpurun_out/t.log
REPS=${REPS:-2} LIBS="${LIBS:-libisim_r1.so libisim.so}" CONFIGS="--config c4" bash tools/ab_libs.sh
