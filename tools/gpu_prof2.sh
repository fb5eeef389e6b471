#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/profile_cfg.sh c4 "--config c4" || exit $?
bash tools/profile_cfg.sh c3 "" || exit $?
