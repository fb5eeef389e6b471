#!/bin/bash
# Kernel-trace stats + bench lines of the other configs (c2 tree, c4 mesh)
# for profiles/<round>/c2, c4 (copy gpurun_out/prof_cfg/<c>/stats/run_kernel_stats.csv, bench.json).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in c2 c4; do
  O=$R/gpurun_out/prof_cfg/$c
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --config $c --no-cpu > $O/b.log 2>&1 || exit 11
  grep "^{\"metric\"" $O/b.log > $O/bench.json || exit 12
done
echo profile configs done
