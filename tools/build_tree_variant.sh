#!/bin/bash
# Build a libisim variant with one lane-tree-walk object (tree.hip for one
# error mode / concurrency pair) recompiled under extra flags:
#   tools/build_tree_variant.sh <out name> <m0c0|m0c1|m1c0|m1c1> <flags...>
# e.g. tools/build_tree_variant.sh libisim_wpe8.so m0c0 -DTREE_WPE2=8
# (run `make -C istio-isotope_amd/csrc` first: the other objects are reused;
# load the variant with ISIM_LIB=istio-isotope_amd/isim/<out name>)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/istio-isotope_amd/csrc
B=$R/build/csrc
OUT=$1; MC=$2; shift 2
mkdir -p $B/variant
HIPFLAGS="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -Wall -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $HIPFLAGS -DTREE_MODEB=${MC:1:1} -DTREE_CONC=${MC:3:1} "$@" -c $C/tree.hip -o $B/variant/tree_$MC.o
objs=""
for o in $B/*.o; do
  [ "$(basename $o)" = "tree_$MC.o" ] && objs="$objs $B/variant/tree_$MC.o" || objs="$objs $o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -o $R/istio-isotope_amd/isim/$OUT $objs
echo built $OUT
