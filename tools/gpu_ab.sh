#!/bin/bash
# Timing A/B of libisim builds on one bench configuration:
#   LIBS="libisim.so libisim_x.so" CFG="--config c4" REPS=2 bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
O=gpurun_out/ab
for rep in $(seq ${REPS:-2}); do for lib in ${LIBS:-libisim.so}; do
  ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 300 python bench.py ${CFG:---config c4} --steps ${STEPS:-5} --warmup 2 --no-cpu --no-mode-b > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 13; }
  python -c "import json;d=json.loads(open('$O/b.log').read().strip().split(chr(10))[-1]);print('$lib', round(d['value']/1e9,4), 'Gtr/s', round(d['roofline']['kernel_ms'],3), 'ms')"
done; done
echo ab done
