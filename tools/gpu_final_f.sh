#!/bin/bash
# final check: full GPU suite, smoke, default bench, N=2 rehearsal at the default batch
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/final/gpu_tests.log; exit 9; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/final/smoke.log; exit 8; }
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench_c3.log 2>&1 || { echo BENCH_FAIL; tail gpurun_out/final/bench_c3.log; exit 7; }
grep '^{' gpurun_out/final/bench_c3.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3', round(d['value']/1e6,2),'Mtr/s', d['roofline']['traffic'], d['roofline']['bytes_per_launch'], d['occupancy']['measured']['mean_waves_per_cu'])"
ISIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/final/n2.log 2>&1 || { echo N2_FAIL; tail -20 gpurun_out/final/n2.log; exit 6; }
grep '^{' gpurun_out/final/n2.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('n2', d['n_gpus'], round(d['value']/1e6,2),'Mtr/s', d['config']['global_batch'])"
echo final F done
