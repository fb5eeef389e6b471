#!/bin/bash
# Same-box A/B of two libisim builds (the current one against $PREV) on bench
# lines (CFGS), alternating, twice: traces/s and ms per step
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lab
O=gpurun_out/lab
PREV=${PREV:-istio-isotope_amd/isim/libisim_prev.so}
for c in ${CFGS:-c4w c3p c3s c4}; do
  for v in prev cur prev cur; do
    if [ $v = prev ]; then export ISIM_LIB=$PREV; else unset ISIM_LIB; fi
    timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu --no-wave-leg $ARGS > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    echo "$c $v $(grep '^{' $O/b.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,2), "M/s", round(d["ms_per_step"],2), "ms")')"
  done
done
