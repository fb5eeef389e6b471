#!/bin/bash
# round 6: k_tiefix's insertion budget per item (8 / 1024 / unbounded) on c5p and c4d
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab
for c in c5p c4d; do
  echo "== $c"
  for lib in libisim.so libisim_tb1024.so libisim_tb1000000000.so; do
    ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/ab/b.log 2>&1 || { tail -5 gpurun_out/ab/b.log; exit 13; }
    python -c "import json;d=json.loads(open('gpurun_out/ab/b.log').read().strip().split(chr(10))[-1]);print('$lib', round(d['value']/1e6,3), 'Mtr/s', round(d['ms_per_step'],2), 'ms')"
  done
done
