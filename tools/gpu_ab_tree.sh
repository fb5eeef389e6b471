#!/bin/bash
# A/B of kind-7 diagnostic builds on config 4
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
REPS=1 LIBS="${LIBS:-libisim_base.so libisim_noasm.so libisim_unroll.so libisim_nosink.so libisim_nohist.so}" CONFIGS="--config c4" bash tools/ab_libs.sh
