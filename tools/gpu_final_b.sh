#!/bin/bash
# Round-end evidence, part B: rocprofv3 kernel-trace stats + PMC passes of c3, c4, c5 and mode B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_cfg.sh c3 "--config c3 --no-mode-b" > gpurun_out/prof_c3.log 2>&1 || { echo PROF_C3_FAIL; tail gpurun_out/prof_c3.log; exit 7; }
echo c3 done
bash tools/profile_c5.sh > gpurun_out/prof_c5.log 2>&1 || { echo PROF_C5_FAIL; tail gpurun_out/prof_c5.log; exit 6; }
echo c5 done
bash tools/profile_cfg.sh c4 "--config c4" > gpurun_out/prof_c4.log 2>&1 || { echo PROF_C4_FAIL; tail gpurun_out/prof_c4.log; exit 5; }
echo c4 done
bash tools/profile_modeb.sh > gpurun_out/prof_b.log 2>&1 || { echo PROF_B_FAIL; tail gpurun_out/prof_b.log; exit 4; }
echo final B done
