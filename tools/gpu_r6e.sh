#!/bin/bash
# round 6: the remaining profile sets (c4w, cdag, c2) and the c4d DES profile
set -o pipefail
cd $GRAFT_REPO_ROOT
SETS="c4w|--config_c4w cdag|--config_cdag c2|--config_c2" bash tools/gpu_r6_prof.sh || exit 7
ISIM_PROF_ROUND=r06 timeout -k 10 900 bash tools/profile_des.sh c4d > gpurun_out/prof_c4d.log 2>&1 || { tail -5 gpurun_out/prof_c4d.log; exit 8; }
echo c4d profiled
