#!/bin/bash
# Profile set of the DES (bench.py --config c5) for profiles/<round>/c5:
#  kernel-trace stats of the default c5 bench, then FETCH_SIZE and WRITE_SIZE
#  in separate PMC passes, then an SQ pass for occupancy; summarised by tools/pmc_summary_c5.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_c5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --config c5 > $O/stats.log 2>&1 || exit 11
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  set -- $p; name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $O/$name.log 2>&1 || exit 12
done
echo profile c5 done
