#!/bin/bash
# Profile set for profiles/<round>/ (run on the GPU box through gpurun):
#  1. rocprofv3 --kernel-trace --stats of the default bench command
#  2. separate PMC passes: FETCH_SIZE | WRITE_SIZE | SQ counters (two passes)
#  3. the Philox4x32-10 throughput ceiling (tools/philox_peak.hip)
# then: python tools/pmc_summary.py gpurun_out/prof <round>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 $R/tools/philox_peak.hip -o $O/philox_peak || exit 10
timeout -k 10 120 $O/philox_peak > $O/philox_peak.json || exit 10
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py > $O/stats.log 2>&1 || exit 11
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" \
         "sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
         "sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  set -- $p; name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/$name.log 2>&1 || exit 12
done
echo profile done
