#!/bin/bash
# one c4d step under rocprofv3 --kernel-trace: the per-dispatch timeline of
# the item engine's passes (tools/c4d_passes.py summarises it per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c4dtr
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o run --output-format csv -- python3 $R/bench.py --config c4d --steps 1 --warmup 1 --no-cpu > $O/bench.log 2>&1 || exit 11
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 $R/tools/c4d_passes.py $f > $O/passes.txt && cat $O/passes.txt | tail -40
gzip -f $f
echo trace done
