#!/bin/bash
# Lane tree walk (kind 7) iteration: its GPU parity tests, then an A/B of
# libisim builds on bench.py --config c4 (phase threshold sweep for the new
# build: ISIM_TREE_PHASE_MIN), then the full-size tests.  Logs: gpurun_out/t7/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/t7
O=gpurun_out/t7
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_walk_gpu.py tests/test_kat_gpu.py tests/test_golden_records_gpu.py -m gpu > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 9; }
tail -1 $O/tests.log
run() {  # lib label extra-env
  env ISIM_LIB=$PWD/istio-isotope_amd/isim/$1 $3 timeout -k 10 300 python bench.py --config c4 --steps ${STEPS:-5} --warmup 2 --no-cpu > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 13; }
  python -c "import json;d=json.loads(open('$O/b.log').read().strip().split(chr(10))[-1]);print('$2', round(d['value']/1e9,3), 'Gtr/s', round(d['roofline']['kernel_ms'],3), 'ms')"
}
for rep in 1 2; do
run libisim_base.so base ""
for T in ${TS:-16 32 48 64}; do run libisim.so new_T$T "ISIM_TREE_PHASE_MIN=$T"; done
done
if [ -z "$NO_FULL" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py -m gpu -s > $O/fullsize.log 2>&1 || { echo FULLSIZE_FAIL; tail -40 $O/fullsize.log; exit 8; }
grep -E "PASSED|FAILED|max_launch" $O/fullsize.log
fi
echo t7 done
