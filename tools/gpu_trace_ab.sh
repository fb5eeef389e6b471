#!/bin/bash
# Per-kernel time of one c5 DES step for several libisim builds:
#   LIBS="libisim_prev.so libisim.so" bash tools/gpu_trace_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for lib in ${LIBS:-libisim_prev.so libisim.so}; do
  O=$R/gpurun_out/trace_ab/${lib%.so}
  mkdir -p $O
  export ISIM_LIB=$R/istio-isotope_amd/isim/$lib
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu ${EXTRA:-} > $O/log 2>&1 || { tail -5 $O/log; exit 11; }
  f=$(find $O -name 'run_kernel_trace.csv' | head -1); cp $f $O/kernel_trace.csv
  echo "== $lib"; python3 $R/tools/trace_show.py $O/kernel_trace.csv
done
