#!/bin/bash
# round 6, final tree: the whole GPU suite as the driver runs it, smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6x
O=gpurun_out/r6x
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -2 $O/smoke.log
