#!/bin/bash
# Profile set of a DES bench line (bench.py --config c5 | c5p | c4d) for
# profiles/<round>/<name>: kernel-trace stats of the default bench line, then
# FETCH_SIZE and WRITE_SIZE in separate PMC passes and an SQ pass for
# occupancy (one untimed + one timed batch each); summarised by
# tools/pmc_summary_des.py.
#   bash tools/profile_des.sh <c5|c5p|c4d>
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=$1
O=$R/gpurun_out/prof_$NAME
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --config $NAME > $O/stats.log 2>&1 || exit 11
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  set -- $p; pn=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc "$@" -d $O/$pn -o run --output-format csv -- python3 $R/bench.py --config $NAME --steps 1 --warmup 1 --no-cpu > $O/$pn.log 2>&1 || exit 12
done
echo profile $NAME done
# summarise on the box (the raw per-dispatch files are too large to copy back)
if [ -n "$ISIM_PROF_ROUND" ]; then
  ISIM_PROF_OUT=$R/gpurun_out/profiles_out python3 $R/tools/pmc_summary_des.py $O $ISIM_PROF_ROUND $NAME > $O/summary.log 2>&1 || exit 13
  rm -rf $O/stats $O/fetch $O/write $O/sq
fi
