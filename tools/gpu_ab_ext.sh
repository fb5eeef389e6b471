#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in libisim_base.so libisim_nosink.so; do for x in 0 1; do
ISIM_TREE_EXT_HBM=$x ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().split(chr(10))[-1]);print('$lib ext_hbm=$x', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', d['config']['launch']['lds_bytes'])"
done; done
