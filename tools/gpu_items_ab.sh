#!/bin/bash
# DES item engine: parity suite, then the c5p / c4d lines of the current
# library against a previous build (ISIM_LIB=$PREV), alternating, twice;
# AB_ENV=NAME: "prev" is the current library with NAME=1 set instead
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/iab
O=gpurun_out/iab
PREV=${PREV:-istio-isotope_amd/isim/libisim_prev.so}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_des_items_gpu.py -m gpu > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 9; }
tail -1 $O/t.log
for c in ${CFGS:-c5p c4d}; do
  for v in prev cur prev cur; do
    if [ -n "$AB_ENV" ]; then
      if [ $v = prev ]; then export $AB_ENV=1; else unset $AB_ENV; fi
    elif [ $v = prev ]; then export ISIM_LIB=$PREV; else unset ISIM_LIB; fi
    timeout -k 10 300 python -u bench.py --config $c --steps 4 --warmup 1 --no-cpu > $O/b.log 2>$O/err.log || { tail -20 $O/err.log; exit 1; }
    echo "$c $v $(grep '^{' $O/b.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms")')"
  done
done
