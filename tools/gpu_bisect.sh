#!/bin/bash
# one DES test against several builds of libisim (ISIM_LIB), for bisecting
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for L in ${LIBS:-libisim.so}; do
  ISIM_LIB=$GRAFT_REPO_ROOT/istio-isotope_amd/isim/$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "${TESTS:-tests/test_des_gpu.py}" -m gpu > gpurun_out/bisect_$L.log 2>&1
  echo "$L rc=$? $(tail -1 gpurun_out/bisect_$L.log)"
done
