#!/bin/bash
# round 6: kind-7 step variants, timing A/B — base (round-6 start), C (one
# Philox block per step, close at the step's end with draws), D (the old
# draws, close at the end with draws), E (one block, every walk closes at the end)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c3p c3s c4w c4; do
  echo "== $c"
  LIBS="libisim_base.so libisim_nc1.so libisim_d.so libisim_e.so" CFG="--config $c" REPS=2 timeout -k 10 400 bash tools/gpu_ab.sh || exit 7
done
