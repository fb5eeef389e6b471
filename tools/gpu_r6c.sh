#!/bin/bash
# round 6: the c4d per-pass dispatch trace, then the first profile sets
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_c4d_trace.sh 2>&1 | tail -60 || exit 5
SETS="c3B|--config_c3_--mode_B_--no-mode-b c3p|--config_c3p c3s|--config_c3s" bash tools/gpu_r6_prof.sh
