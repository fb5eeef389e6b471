#!/bin/bash
# round 6, final lines: every bench configuration once (c3 with its mode-B
# legs, c1, c2, c5, c5p, c4d), the N=2 gloo rehearsal, the c3 profile set
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6s
O=gpurun_out/r6s
for c in c3 c1 c2 c5 c5p c4d; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['ms_per_step'], {k:(d[k]['value'],d[k].get('kernel_kind')) for k in ('mode_b','mode_b_informative') if k in d})"
done
ISIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --config c3 --mode-b-steps 2 > $O/n2.log 2>&1 || { echo "N2 FAIL"; tail -30 $O/n2.log; exit 5; }
grep '^{' $O/n2.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('n2 c3', d['n_gpus'], round(d['value']/1e6,2), 'Mtr/s')"
SETS="c3|--config_c3_--no-mode-b" bash tools/gpu_r6_prof.sh
