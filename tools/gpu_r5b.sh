#!/bin/bash
# Round 5, GPU session B: the u64 lane tree walk (kind 7 with u64 time) —
# its parity tests, then the c3s bench line (with the wave-interpreter leg)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5b
O=gpurun_out/r5b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_fullsize_gpu.py tests/test_des_items_gpu.py -k "u64 or sequential_probability or kat or config3s or t64 or c3s or reference_topologies" -m gpu > $O/t.log 2>&1 || { echo T_FAIL; grep -E "FAILED|Error" $O/t.log | head; tail -30 $O/t.log; exit 9; }
tail -1 $O/t.log
timeout -k 10 400 python bench.py --config c3s --no-cpu --steps 5 > $O/c3s.log 2>&1 || { echo C3S_FAIL; tail $O/c3s.log; exit 7; }
grep '^{' $O/c3s.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3s', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms wave', round(d['wave_walk']['value']/1e6,3), 'x', round(d['speedup_vs_wave_walk'],1), 'hops', round(d['config']['hop_visits_per_trace'],1))"
echo done
