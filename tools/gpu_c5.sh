set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/c5.log 2>&1 || { tail -20 gpurun_out/c5.log; exit 1; }
tail -1 gpurun_out/c5.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c5prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/c5prof.log 2>&1 || exit 2
find $GRAFT_REPO_ROOT/gpurun_out/c5prof -name "*kernel_stats.csv" -exec head -12 {} \;
