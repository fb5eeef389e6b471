#!/bin/bash
# A/B of the statistics pass's items per lane (k_qout / k_fin) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in ${CFGS:-c5p c4d}; do
  for v in 16 4 8 2 16; do
    ISIM_DES_ITEMS_STATS_SPAN=$v timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    echo "$c span $v $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
  done
done
