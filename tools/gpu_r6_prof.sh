#!/bin/bash
# round 6 profile sets (tools/profile_cfg.sh: rocprofv3 --kernel-trace --stats
# of the bench line + separate FETCH / WRITE / SQ PMC passes) of the configs
# whose kernels changed this round; summarised here by tools/pmc_summary.py
set -o pipefail
cd $GRAFT_REPO_ROOT
for spec in "c3B|--config c3 --mode B --no-mode-b" "c3p|--config c3p" "c3s|--config c3s" "c4w|--config c4w" \
            "cdag|--config cdag" "c2|--config c2" ${EXTRA}; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 900 bash tools/profile_cfg.sh $name "$args" > gpurun_out/prof_$name.log 2>&1 || { echo "$name profile failed"; tail -5 gpurun_out/prof_$name.log; exit 7; }
  echo "$name profiled"
done
echo prof done
