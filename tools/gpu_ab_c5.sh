#!/bin/bash
# A/B of libisim builds on bench.py --config c5 (timing only; build variants in-tree first)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for rep in 1 2; do for lib in ${LIBS:-libisim.so}; do
ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu $1 > gpurun_out/c5ab.log 2>&1 || { tail -5 gpurun_out/c5ab.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/c5ab.log').read().strip().split(chr(10))[-1]);print('$lib', round(d['value']/1e6,3), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', round(d['roofline']['frac'],3))"
done; done
