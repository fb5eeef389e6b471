#!/bin/bash
# DES parity suite on a libisim variant (ISIM_LIB), then c5 timing A/B against
# the default build:  LIBS="libisim_hoist.so" bash tools/gpu_des_variant.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/desv
O=gpurun_out/desv
for lib in ${LIBS:-libisim_hoist.so}; do
  ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_des_gpu.py tests/test_golden_records_gpu.py -m gpu > $O/tests_$lib.log 2>&1 && echo "$lib DES tests: $(tail -1 $O/tests_$lib.log)" || { echo "$lib DES TESTS FAIL"; grep -E "FAILED|Error|assert" $O/tests_$lib.log | head -20; tail -5 $O/tests_$lib.log; }
done
if [ -n "$AB" ]; then
for rep in 1 2; do for lib in libisim.so ${LIBS:-libisim_hoist.so}; do
  ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 13; }
  python -c "import json;d=json.loads(open('$O/c5.log').read().strip().split(chr(10))[-1]);print('$lib', round(d['value']/1e6,3), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', round(d['roofline']['frac'],3))"
done; done
fi
echo desv done
