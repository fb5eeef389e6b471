#!/bin/bash
# Per-dispatch kernel trace of one DES step (bench.py --config c5): which
# des_* launches of a step take the time (tools/trace_show.py summarises).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_c5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 1 --no-cpu ${EXTRA:-} > $O/log 2>&1 || exit 11
f=$(find $O -name 'run_kernel_trace.csv' | head -1); cp $f $O/kernel_trace.csv
echo trace done
