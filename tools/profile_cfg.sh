#!/bin/bash
# Profile set of one bench configuration (run on the GPU box through gpurun):
#   bash tools/profile_cfg.sh <name> "<bench args>"
#  1. rocprofv3 --kernel-trace --stats of the bench command
#  2. separate PMC passes: FETCH_SIZE | WRITE_SIZE | SQ counters (two passes)
#     | VALU lane activity (optional: a failing pass does not stop the set)
# then, here: python tools/pmc_summary.py gpurun_out/prof_<name> <round> <name>
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=$1
ARGS=$2
O=$R/gpurun_out/prof_$NAME
mkdir -p $O
echo "$ARGS" > $O/args
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/stats.log 2>&1 || exit 11
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" \
         "sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
         "sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  set -- $p; name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 3 --warmup 1 --no-cpu > $O/$name.log 2>&1 || exit 12
done
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/sq3 -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 3 --warmup 1 --no-cpu > $O/sq3.log 2>&1 || echo "sq3 pass failed (optional)"
echo profile done
