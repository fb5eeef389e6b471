#!/bin/bash
# Kind-7 (lane tree walk) check on the box: the GPU parity suites that run the
# tree walk, then short bench lines of config 4 and c3p (probabilities in
# $PROBS).  Logs under gpurun_out/tree/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tree
O=gpurun_out/tree
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_golden_records_gpu.py -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 9; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4.log 2>&1 || { echo BENCH_c4_FAIL; tail -20 $O/bench_c4.log; exit 6; }
grep '^{' $O/bench_c4.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4', round(d['value']/1e9,3),'Gtr/s', round(d['roofline']['kernel_ms'],3),'ms', d['config']['launch'])"
for p in ${PROBS:-50}; do
timeout -k 10 300 python bench.py --config c3p --prob $p --steps 5 --warmup 2 --no-cpu > $O/bench_c3p$p.log 2>&1 || { echo BENCH_c3p_FAIL; tail -20 $O/bench_c3p$p.log; exit 5; }
grep '^{' $O/bench_c3p$p.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3p$p', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms hops/trace', round(d['config']['hop_visits_per_trace'],1), 'wave', round(d['wave_walk']['value']/1e6,2), 'x', round(d['speedup_vs_wave_walk'],2), d['config']['launch'])"
done
echo tree done
