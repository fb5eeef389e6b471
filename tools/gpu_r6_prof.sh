#!/bin/bash
# round 6 profile sets (tools/profile_cfg.sh: rocprofv3 --kernel-trace --stats
# of the bench line + separate FETCH / WRITE / SQ PMC passes) of the configs
# whose kernels changed this round; summarised here by tools/pmc_summary.py
set -o pipefail
cd $GRAFT_REPO_ROOT
# SETS: the profile sets of this call (each name|bench args); default: every changed config
SETS=${SETS:-"c3B|--config_c3_--mode_B_--no-mode-b c3p|--config_c3p c3s|--config_c3s c4w|--config_c4w cdag|--config_cdag c2|--config_c2"}
for spec in $SETS; do
  spec=${spec//_/ }
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 900 bash tools/profile_cfg.sh $name "$args" > gpurun_out/prof_$name.log 2>&1 || { echo "$name profile failed"; tail -5 gpurun_out/prof_$name.log; exit 7; }
  echo "$name profiled"
done
echo prof done
