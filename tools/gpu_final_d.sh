#!/bin/bash
# bench lines at the 2^24 default batch + c3/c4 profile sets + mode-B stats
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py > gpurun_out/final/bench_c3.log 2>&1 || { echo BENCH_FAIL; tail gpurun_out/final/bench_c3.log; exit 7; }
timeout -k 10 600 python bench.py --config c4 > gpurun_out/final/bench_c4.log 2>&1 || { echo BENCH_C4_FAIL; exit 7; }
bash tools/profile_cfg.sh c3 "--config c3 --no-mode-b" > gpurun_out/prof_c3.log 2>&1 || { echo PROF_C3_FAIL; tail gpurun_out/prof_c3.log; exit 6; }
bash tools/profile_cfg.sh c4 "--config c4" > gpurun_out/prof_c4.log 2>&1 || { echo PROF_C4_FAIL; tail gpurun_out/prof_c4.log; exit 5; }
bash tools/profile_modeb.sh > gpurun_out/prof_b.log 2>&1 || { echo PROF_B_FAIL; exit 4; }
for c in c3 c4; do grep '^{' gpurun_out/final/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms', d['config']['global_batch'])"; done
echo final D done
