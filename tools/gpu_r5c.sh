#!/bin/bash
# Round 5, GPU session C: the DES item engine with incremental quiet passes —
# its parity suite, then c4d (and c5p) bench lines, incremental vs every item
# per pass (ISIM_DES_ITEMS_NO_INCR)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5c
O=gpurun_out/r5c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_des_items_gpu.py -m gpu > $O/t.log 2>&1 || { echo T_FAIL; grep -E "FAILED|Error" $O/t.log | head; tail -30 $O/t.log; exit 9; }
tail -1 $O/t.log
for v in "" "ISIM_DES_ITEMS_NO_INCR=1"; do
  timeout -k 10 400 env $v ISIM_DES_DEBUG=1 python bench.py --config c4d --no-cpu --steps 2 --warmup 1 > $O/c4d_$v.log 2>&1 || { echo C4D_FAIL $v; tail $O/c4d_$v.log; exit 7; }
  grep '^{' $O/c4d_$v.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c4d [$v]', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],1),'ms')"
  grep "cyclic schedule" $O/c4d_$v.log | tail -1
done
echo done
