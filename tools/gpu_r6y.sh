#!/bin/bash
# round 6: two-workgroup kind-7 kernels at 8 waves per SIMD (TREE_WPE2=8, 64 VGPRs) vs 6
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c4 c1; do
  echo "== $c"
  LIBS="libisim.so libisim_w8.so" CFG="--config $c" REPS=2 timeout -k 10 300 bash tools/gpu_ab.sh || exit 7
done
