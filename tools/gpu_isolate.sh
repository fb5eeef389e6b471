#!/bin/bash
# one failing item-engine case under each A/B switch of des_items.hip
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/iso
T=${T:-"tests/test_des_items_gpu.py::test_items_match_event_oracle[zero_hold_mix-300000]"}
for v in NONE ISIM_DES_ITEMS_TWO_SORTS ISIM_DES_ITEMS_NO_ORDER_REUSE ISIM_DES_ITEMS_NO_SKIP ISIM_DES_ITEMS_FAT_QUIET; do
  env $v=1 timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread "$T" > gpurun_out/iso/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -E 'records differ|passed|failed' gpurun_out/iso/$v.log | head -2 | tr '\n' ' ')"
  [ $rc -gt 1 ] && exit $rc
done
exit 0
