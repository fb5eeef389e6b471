#!/bin/bash
# Same-box A/B: c4d under the previous commit's library vs the current one
# (no debug output), c5p slab caps vs two walks, and the lane tree walk's
# scans per macro step (TW_SCAN variants) on c3p / config 4
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab5
O=gpurun_out/ab5
line() { grep '^{' $O/b.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"]/1e6,3), "M/s", round(d["ms_per_step"],2), "ms")'; }
# run <tag> <config> [NAME=value ...]
run() { local tag=$1 cfg=$2; shift 2
  timeout -k 10 300 env X=1 "$@" python -u bench.py --config $cfg --steps 4 --warmup 1 --no-cpu --no-wave-leg > $O/b.log 2>$O/err.log || { echo FAIL $tag; tail -5 $O/err.log; return 1; }
  echo "$tag $(line)"; }
P=ISIM_LIB=istio-isotope_amd/isim/libisim_prev.so
for i in 1 2; do
  run "c4d prev" c4d $P || exit 1
  run "c4d cur" c4d || exit 1
done
run "c5p two" c5p ISIM_DES_ITEMS_TWO_WALKS=1 || exit 1
for v in 1024 2048 512; do run "c5p cap$v" c5p ISIM_DES_ITEMS_SLAB_CAP=$v || exit 1; done
run "c5p prev" c5p $P || exit 1
for l in libisim libisim_scan5 libisim_scan8 libisim; do
  run "c3p $l" c3p ISIM_LIB=istio-isotope_amd/isim/$l.so || exit 1
  run "c4 $l" c4 ISIM_LIB=istio-isotope_amd/isim/$l.so || exit 1
done
echo ab done
