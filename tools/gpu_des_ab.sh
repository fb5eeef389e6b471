#!/bin/bash
# DES variants: DES parity suite (TESTS=0 skips it), then config-5 timing of
# "label:library:ENV=value,..." runs, REPS times (the round-3 treelet A/B,
# DESIGN.md §10.7, ran as RUNS="prev:libisim_prev.so: on:libisim.so:ISIM_DES_TREELET=1 ..."):
#   RUNS="prev:libisim_prev.so: new:libisim.so:" bash tools/gpu_des_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dest
O=gpurun_out/dest
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_des_gpu.py tests/test_golden_records_gpu.py -m gpu > $O/tests.log 2>&1 && echo "DES tests: $(tail -1 $O/tests.log)" || { echo "DES TESTS FAIL"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 9; }
fi
RUNS=${RUNS:-"prev:libisim_prev.so: new:libisim.so:"}
for rep in $(seq ${REPS:-2}); do
for r in $RUNS; do
  IFS=: read label lib envs <<< "$r"
  env ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib ${envs//,/ } timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 13; }
  python -c "import json;d=json.loads(open('$O/c5.log').read().strip().split(chr(10))[-1]);print('$label', round(d['value']/1e6,3), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', round(d['roofline']['frac'],3))"
done; done
echo dest done
