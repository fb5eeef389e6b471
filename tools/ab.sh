#!/bin/bash
# A/B libraries: ISIM_LIB=<lib> bench.py, prints value per lib (repeat 2x interleaved)
mkdir -p gpurun_out
for rep in 1 2; do
for L in istio-isotope_amd/isim/libisim.so "$@"; do
  ISIM_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/b.log 2>&1 || { cat gpurun_out/b.log | tail -5; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().split(chr(10))[-1]);print('$L', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],2), 'ms', d['config']['launch']['blocks_per_cu'])"
done; done
