#!/bin/bash
# Kernel-trace stats of the mode-B config-3 bench (close-list kernel, kind 6)
# for profiles/<round>/c3_modeB (copy gpurun_out/prof_b/stats/*kernel_stats.csv and b.json).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --config c3 --mode B --no-cpu > $O/b.log 2>&1 || exit 11
grep "^{\"metric\"" $O/b.log > $O/b.json
echo profile mode B done
