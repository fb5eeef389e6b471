#!/bin/bash
# One PMC pass per mode of the stream kernel: instruction mix and issue activity.
#   bash tools/pmc_quick.sh "<bench args>" ...   (run on the GPU box through gpurun)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/p$i -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu $a > $O/p$i.log 2>&1 || exit 12
  echo "$a" > $O/p$i.args
done
echo pmc done
