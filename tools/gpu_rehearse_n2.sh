#!/bin/bash
# N=2 rehearsal of bench.py's multi-rank flow on ONE GPU: two ranks share cuda:0,
# gloo instead of RCCL (the RCCL communicator needs distinct GPUs)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in ${CFGS_N2:-"--config c3 --no-mode-b" "--config c5 --batch 65536" "--config c3 --mode-b-steps 2" "--config c5p --batch 65536" "--config c4d --batch 262144"}; do
ISIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 $cfg > gpurun_out/n2.log 2>&1 || { echo "N2 FAIL: $cfg"; tail -30 gpurun_out/n2.log; exit 5; }
grep '^{' gpurun_out/n2.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg', d['n_gpus'], round(d['value']/1e6,2), 'Mtr/s', d['config']['merge'], d['config']['global_batch'], d.get('n_500_frac'))"
done
echo n2 done
