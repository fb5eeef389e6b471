#!/bin/bash
# Round-end evidence, part B (run BEFORE part A, so the bench lines read the
# fresh summaries): rocprofv3 kernel-trace stats + PMC passes of c3 (mode A),
# c3 mode B, c4, c1 and c5.  Then, here:
#   python tools/pmc_summary.py gpurun_out/prof_<name> <round> <name>   (c3 c3B c4 c1)
#   python tools/pmc_summary_c5.py gpurun_out/prof_c5 <round>
set -o pipefail
cd $GRAFT_REPO_ROOT
prof() {  # name "bench args" exit-code
  bash tools/profile_cfg.sh $1 "$2" > gpurun_out/prof_$1.log 2>&1 || { echo PROF_$1_FAIL; tail gpurun_out/prof_$1.log; exit $3; }
  echo $1 done
}
prof c3 "--config c3 --no-mode-b" 7
prof c3B "--config c3 --mode B --no-mode-b" 6
prof c4 "--config c4" 5
prof c1 "--config c1" 4
bash tools/profile_c5.sh > gpurun_out/prof_c5.log 2>&1 || { echo PROF_C5_FAIL; tail gpurun_out/prof_c5.log; exit 3; }
echo final B done
