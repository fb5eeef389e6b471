#!/bin/bash
# The DES item engine on the GPU box (through gpurun): parity tests, short
# bench lines of the dynamic-walk DES configurations and a kernel-trace
# profile of each (per-kernel time).
#   CFGS="c5p c4d" TESTS=1 PROF=1 bash tools/gpu_items.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/items
mkdir -p $O
cd $R
if [ "${TESTS:-1}" = 1 ]; then
  ISIM_DES_DEBUG=1 timeout -k 10 600 python -u -m pytest tests/test_des_items_gpu.py -q --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for c in ${CFGS:-c5p c4d}; do
  ISIM_DES_DEBUG=1 timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:---no-cpu} \
    > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 $O/bench_$c.log; exit 2; }
  grep '^{' $O/bench_$c.log | tail -1
  if [ "${PROF:-1}" = 1 ]; then
    # the kernel trace itself is large (thousands of launches per step): only the stats come back
    P=/tmp/items_prof_$c
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P -o run \
      --output-format csv -- python3 $R/bench.py --config $c --steps 2 --warmup 1 --no-cpu > $O/prof_$c.log 2>&1) \
      || { echo "profile $c failed"; tail -20 $O/prof_$c.log; exit 3; }
    find $P -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_$c.csv \;
    head -25 $O/kernel_stats_$c.csv | cut -d, -f1-8
  fi
done
echo items done
