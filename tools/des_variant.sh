#!/bin/bash
# Build libisim variants that differ only in des.hip compile-time knobs:
#   tools/des_variant.sh NAME -DISIM_DES_CHAIN_BELOW=0 ...
# -> istio-isotope_amd/isim/libisim_NAME.so (A/B with tools/ab_libs.sh, LIBS=...)
set -e
cd "$(dirname "$0")/../istio-isotope_amd/csrc"
make -s
name=$1; shift
B=../../build/csrc
mkdir -p ../../build/v
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -Wall \
  -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c des.hip -o ../../build/v/des_$name.o
objs=$(ls $B/*.o | grep -v '/des.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib -o ../isim/libisim_$name.so $objs ../../build/v/des_$name.o
echo built libisim_$name.so
