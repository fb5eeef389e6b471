#!/bin/bash
# Round-end evidence, part B (run BEFORE part A, so the bench lines read the
# fresh summaries): rocprofv3 kernel-trace stats + PMC passes of the profiles
# named in PROFS (default: c3 c3B c4 c3p c3s c4w c1 via profile_cfg.sh, then the
# DES lines c5 c5p c4d via profile_des.sh, summarised on the box into
# gpurun_out/profiles_out/).  Then, here:
#   python tools/pmc_summary.py gpurun_out/prof_<name> <round> <name>   (c3 c3B c4 c3p c3s c4w c1)
#   cp -r gpurun_out/profiles_out/* profiles/                            (c5 c5p c4d)
set -o pipefail
cd $GRAFT_REPO_ROOT
export ISIM_PROF_ROUND=${ISIM_PROF_ROUND:-r05}
for name in ${PROFS:-c3 c3B c4 c3p c3s c4w c1 c5 c5p c4d}; do
  case $name in
    c3) args="--config c3 --no-mode-b" ;;
    c3B) args="--config c3 --mode B --no-mode-b" ;;
    c3p|c3s|c4w) args="--config $name --no-wave-leg" ;;
    c5|c5p|c4d) bash tools/profile_des.sh $name > gpurun_out/prof_$name.log 2>&1 || { echo PROF_${name}_FAIL; tail gpurun_out/prof_$name.log; exit 3; }
        echo $name done; continue ;;
    *) args="--config $name" ;;
  esac
  bash tools/profile_cfg.sh $name "$args" > gpurun_out/prof_$name.log 2>&1 || { echo PROF_${name}_FAIL; tail gpurun_out/prof_$name.log; exit 4; }
  echo $name done
done
echo final B done
