#!/bin/bash
# config-3 throughput against the batch length (traces per launch)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in 4194304 8388608 16777216 4194304; do
timeout -k 10 300 python bench.py --config c3 --no-mode-b --no-cpu --steps 5 --warmup 2 --batch $b > gpurun_out/c3b.log 2>&1 || { tail -5 gpurun_out/c3b.log; exit 13; }
grep '^{' gpurun_out/c3b.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print($b, round(d['value']/1e6,2),'Mtr/s', round(d['ms_per_step'],3),'ms/step', round(d['roofline']['kernel_ms'],3))"
done
