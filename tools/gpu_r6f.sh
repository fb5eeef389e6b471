#!/bin/bash
# round 6: the whole GPU suite as the driver runs it, then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6f
O=gpurun_out/r6f
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -4 $O/smoke.log
ISIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --config c3 --mode-b-steps 2 > $O/n2.log 2>&1 || { echo "N2 FAIL"; tail -30 $O/n2.log; exit 5; }
grep '^{' $O/n2.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('n2 c3', d['n_gpus'], round(d['value']/1e6,2), 'Mtr/s', d['config']['merge'], d['mode_b']['kernel_kind'])"
