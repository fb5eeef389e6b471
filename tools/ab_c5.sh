#!/bin/bash
# DES parity + c5 bench line (one gpurun call)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_des_gpu.py -m gpu > gpurun_out/des_tests.log 2>&1 || { tail -30 gpurun_out/des_tests.log; exit 12; }
tail -1 gpurun_out/des_tests.log
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu > gpurun_out/c5.log 2>&1 || { tail -5 gpurun_out/c5.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/c5.log').read().strip().split(chr(10))[-1]);print('c5', round(d['value']/1e6,3), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', round(d['roofline']['frac'],3))"
