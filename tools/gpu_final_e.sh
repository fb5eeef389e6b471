#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py --config c4 > gpurun_out/final/bench_c4.log 2>&1 || { echo BENCH_C4_FAIL; tail gpurun_out/final/bench_c4.log; exit 7; }
bash tools/profile_cfg.sh c4 "--config c4" > gpurun_out/prof_c4.log 2>&1 || { echo PROF_C4_FAIL; tail gpurun_out/prof_c4.log; exit 5; }
grep '^{' gpurun_out/final/bench_c4.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms', d['config']['global_batch'])"
echo final E done
