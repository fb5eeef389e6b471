#!/bin/bash
# Build a libisim variant with one HIP source recompiled under extra flags:
#   tools/build_variant.sh <out name> <source.hip> <flags...>
# e.g. tools/build_variant.sh libisim_hoist.so des.hip -DDES_HOIST_500
# (run `make -C istio-isotope_amd/csrc` first: the other objects are reused)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/istio-isotope_amd/csrc
B=$R/build/csrc
OUT=$1; SRC=$2; shift 2
mkdir -p $B/variant
HIPFLAGS="-O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -Wall -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c $C/$SRC -o $B/variant/${SRC%.hip}.o
objs=""
for o in $B/*.o; do
  [ "$(basename $o)" = "${SRC%.hip}.o" ] && objs="$objs $B/variant/${SRC%.hip}.o" || objs="$objs $o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -o $R/istio-isotope_amd/isim/$OUT $objs
echo built $OUT
