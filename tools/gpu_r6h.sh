#!/bin/bash
# round 6: the workgroup flush's share of kind-7 launches (timing A/B against
# a build with the flush compiled out, TREE_NO_FLUSH)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c3p c3s c4 c4w; do
  echo "== $c"
  LIBS="libisim.so libisim_noflush.so" CFG="--config $c" REPS=2 timeout -k 10 400 bash tools/gpu_ab.sh || exit 7
done
