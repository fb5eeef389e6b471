#!/bin/bash
# Round-end evidence, part B (run BEFORE part A, so the bench lines read the
# fresh summaries): rocprofv3 kernel-trace stats + PMC passes of the profiles
# named in PROFS (default all: c3 c3B c4 c3p c1 c5; c3B = config 3 in mode B).
# Then, here:
#   python tools/pmc_summary.py gpurun_out/prof_<name> <round> <name>   (c3 c3B c4 c3p c1)
#   python tools/pmc_summary_c5.py gpurun_out/prof_c5 <round>
set -o pipefail
cd $GRAFT_REPO_ROOT
for name in ${PROFS:-c3 c3B c4 c3p c1 c5}; do
  case $name in
    c3) args="--config c3 --no-mode-b" ;;
    c3B) args="--config c3 --mode B --no-mode-b" ;;
    c3p) args="--config c3p --no-wave-leg" ;;
    c5) bash tools/profile_c5.sh > gpurun_out/prof_c5.log 2>&1 || { echo PROF_c5_FAIL; tail gpurun_out/prof_c5.log; exit 3; }
        echo c5 done; continue ;;
    *) args="--config $name" ;;
  esac
  bash tools/profile_cfg.sh $name "$args" > gpurun_out/prof_$name.log 2>&1 || { echo PROF_${name}_FAIL; tail gpurun_out/prof_$name.log; exit 4; }
  echo $name done
done
echo final B done
