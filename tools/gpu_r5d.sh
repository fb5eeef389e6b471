#!/bin/bash
# Round 5, GPU session D: kind-7 parity (both LDS row formats) + item engine,
# then A/B: config 4 and c3p with wide vs compact LDS rows; c4d bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5d
O=gpurun_out/r5d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_des_items_gpu.py tests/test_golden_records_gpu.py -m gpu > $O/t.log 2>&1 || { echo T_FAIL; grep -E "FAILED|Error" $O/t.log | head; tail -30 $O/t.log; exit 9; }
tail -1 $O/t.log
ISIM_TREE_COMPACT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_gpu.py tests/test_kat_gpu.py -m gpu > $O/tc.log 2>&1 || { echo TC_FAIL; grep -E "FAILED|Error" $O/tc.log | head; tail -30 $O/tc.log; exit 9; }
tail -1 $O/tc.log
bash tools/gpu_tree_ab.sh "c4" "c4 ISIM_TREE_COMPACT=1" "c4" "c4 ISIM_TREE_COMPACT=1" "c3p" "c3p ISIM_TREE_WIDE=1" "c3p ISIM_TREE_WIDE=1 ISIM_TREE_NODES_LDS=1" || exit 8
timeout -k 10 400 python bench.py --config c4d --no-cpu --steps 3 --warmup 1 > $O/c4d.log 2>&1 || { echo C4D_FAIL; tail $O/c4d.log; exit 7; }
grep '^{' $O/c4d.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4d', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],1),'ms')"
echo done
