#!/bin/bash
# A/B timing of lane-tree-walk variants: bench lines of config 4 and c3p under
# environment settings / variant libraries (tools/build_tree_variant.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tree
O=gpurun_out/tree
# a spec: <config> [NAME=value ...] [--bench-arg ...]
ab() { local cfg=$1; shift
  local envs=() args=()
  for a in "$@"; do case "$a" in --*) args+=("$a");; *) envs+=("$a");; esac; done
  timeout -k 10 200 env "${envs[@]}" python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu --no-wave-leg "${args[@]}" > $O/ab.log 2>&1 || { echo AB_FAIL $cfg "$@"; tail -5 $O/ab.log; return 1; }
  grep '^{' $O/ab.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg $*', round(d['value']/1e9,4), 'Gtr/s', round(d['roofline']['kernel_ms'],3), 'ms', d['config']['launch']['wg_threads'], d['config']['launch']['blocks_per_cu'], d['config']['launch']['lds_bytes'])"; }
for spec in "${@}"; do ab $spec || exit 10; done
echo ab done
