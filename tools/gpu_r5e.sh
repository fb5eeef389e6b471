#!/bin/bash
# Round 5, GPU session E: item-engine parity, c4d bench (+ passes/syncs), c4d kernel split
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5e
O=gpurun_out/r5e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_des_items_gpu.py tests/test_des_gpu.py -m gpu > $O/t.log 2>&1 || { echo T_FAIL; grep -E "FAILED|Error" $O/t.log | head; tail -30 $O/t.log; exit 9; }
tail -1 $O/t.log
for c in c4d c5p; do
timeout -k 10 400 python bench.py --config $c --no-cpu --steps 3 --warmup 1 > $O/$c.log 2>&1 || { echo ${c}_FAIL; tail $O/$c.log; exit 7; }
grep '^{' $O/$c.log | python -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];print('$c', round(d['value']/1e6,2),'Mtr/s', round(d['roofline']['kernel_ms'],1),'ms passes', c.get('des_passes_per_step'), 'syncs', c.get('des_syncs_per_step'))"
done
echo done
