#!/bin/bash
# GPU parity suite + config sweep (one gpurun call)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 9; }
tail -2 gpurun_out/gpu_tests.log
for a in "--config c3" "--config c4 --batch 1048576" "--config c4 --batch 1048576 --no-svc-dur" "--config c3 --mode B" "--config c2"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $a > gpurun_out/sweep.log 2>&1 || { echo BENCH_FAIL $a; tail -5 gpurun_out/sweep.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sweep.log').read().strip().split(chr(10))[-1]);print('$a', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms')"
done
