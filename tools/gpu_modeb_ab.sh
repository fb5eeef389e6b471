#!/bin/bash
# Mode B (kernel kind 6) A/B: the default c3 line with its mode-B legs under
# the current library and a variant (ISIM_LIB), twice each; then the mode-B
# parity tests of the current library
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/mb
O=gpurun_out/mb
VAR=${VAR:-istio-isotope_amd/isim/libisim_oldwalk.so}
for rep in 1 2; do
for lib in "" "$VAR"; do
  timeout -k 10 300 env ${lib:+ISIM_LIB=$lib} python bench.py --no-cpu --steps 5 --warmup 2 --mode-b-steps 5 > $O/b.log 2>&1 || { echo B_FAIL $lib; tail $O/b.log; exit 7; }
  grep '^{' $O/b.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('[${lib:-current}]', 'A', round(d['value']/1e6,1), 'B', round(d['mode_b']['value']/1e6,1), 'ratio', round(d['mode_b']['value']/d['value'],3), 'Binf', round(d['mode_b_informative']['value']/1e6,1), 'kms', round(d['mode_b']['kernel_ms'],2))"
done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_gpu.py tests/test_fullsize_gpu.py tests/test_kat_gpu.py tests/test_golden_records_gpu.py -k "mode_b or close_list or stream or config3 or kat or golden or reference" -m gpu > $O/t.log 2>&1 || { echo T_FAIL; grep -E "FAILED|Error" $O/t.log | head; tail -20 $O/t.log; exit 9; }
tail -1 $O/t.log
echo done
