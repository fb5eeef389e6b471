#!/bin/bash
# quick GPU check: walk parity tests + bench lines (args: extra bench configs, ';'-separated)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_walk_gpu.py tests/test_fullsize_gpu.py -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 12; }
tail -1 gpurun_out/t.log
IFS=';' read -ra CFGS <<< "${1:---config c3;--config c3 --mode B}"
for a in "${CFGS[@]}"; do
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $a > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().split(chr(10))[-1]);print('$a', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', d.get('compute_roofline') and round(d['compute_roofline']['frac'],3))"
done
