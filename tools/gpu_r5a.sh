#!/bin/bash
# Round 5, first GPU session: the new parity tests, the whole -m gpu suite,
# then c3p with the compact LDS rows (nodes in global memory, every row in
# LDS) against nodes in LDS (ISIM_TREE_NODES_LDS), and config 4.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5a
O=gpurun_out/r5a
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_des_items_gpu.py tests/test_walk_gpu.py -k "zero_hold or bench_graph or c4d_bench_batch or spill_two" -m gpu > $O/new.log 2>&1 || { echo NEW_FAIL; tail -40 $O/new.log; exit 9; }
grep -E "PASSED|FAILED" $O/new.log | sed 's/.*:://' | tr '\n' ' '; echo
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/all.log 2>&1 || { echo ALL_FAIL; tail -30 $O/all.log; exit 8; }
tail -1 $O/all.log
for v in "" "ISIM_TREE_NODES_LDS=1"; do
  env $v timeout -k 10 300 python bench.py --config c3p --no-wave-leg --no-cpu --steps 5 > $O/c3p_$v.log 2>&1 || { echo C3P_FAIL $v; tail $O/c3p_$v.log; exit 7; }
  grep '^{' $O/c3p_$v.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3p [$v]', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms')"
done
timeout -k 10 300 python bench.py --config c4 --no-cpu --steps 5 > $O/c4.log 2>&1 || { echo C4_FAIL; tail $O/c4.log; exit 6; }
grep '^{' $O/c4.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],3),'ms')"
echo done
