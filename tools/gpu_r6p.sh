#!/bin/bash
# round 6: the close's reads issued before the scans (TW_CLOSE_PREFETCH,
# libisim_cp.so) — timing A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c3p c3s c4w c4 cdag; do
  echo "== $c"
  LIBS="libisim.so libisim_cp.so" CFG="--config $c" REPS=2 timeout -k 10 300 bash tools/gpu_ab.sh || exit 7
done
