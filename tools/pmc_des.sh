#!/bin/bash
# Per-dispatch instruction mix of one DES step (bench.py --config c5):
#   python tools/pmc_des_show.py gpurun_out/pmc_des
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_des
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $O/p1 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 1 --no-cpu > $O/p1.log 2>&1 || exit 12
timeout -k 10 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/p2 -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 1 --warmup 1 --no-cpu > $O/p2.log 2>&1 || exit 12
echo pmc des done
