#!/bin/bash
# round 6: register frames of the narrow spilling kernels (8 / 6 / 4,
# ISIM_TREE_SPILL_REGS) — timing A/B on c3p and c3s, then their parity at the bench batch
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6r
for c in c3p c3s; do
  echo "== $c"
  LIBS="libisim.so libisim_sr6.so libisim_sr4.so" CFG="--config $c" REPS=2 timeout -k 10 300 bash tools/gpu_ab.sh || exit 7
done
