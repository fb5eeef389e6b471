#!/bin/bash
# kind 7 (lane tree walk): parity on the walk + KAT + full-size tests, then the c4 bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
$T 300 $PT tests/test_walk_gpu.py -m gpu -k "mesh or probability or tree or wave or refill" > gpurun_out/tree1.log 2>&1 || { tail -40 gpurun_out/tree1.log; exit 11; }
tail -1 gpurun_out/tree1.log
$T 300 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu > gpurun_out/b_c4.log 2>&1 || { tail -5 gpurun_out/b_c4.log; exit 13; }
tail -1 gpurun_out/b_c4.log
$T 600 $PT tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_fullsize_gpu.py -m gpu > gpurun_out/tree2.log 2>&1 || { tail -40 gpurun_out/tree2.log; exit 12; }
tail -1 gpurun_out/tree2.log
