#!/bin/bash
# Kind-7 bench-batch parity tests, then the profile sets of config 4 and c3p
# (tools/profile_cfg.sh).  Logs under gpurun_out/tree/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tree
O=gpurun_out/tree
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_fullsize_gpu.py -m gpu -k "config4_bench_batch or config3p or guarded" > $O/fullsize.log 2>&1 || { echo FULLSIZE_FAIL; grep -E "PASS|FAIL|Error|assert" $O/fullsize.log | tail -20; exit 9; }
grep -E "PASSED|FAILED" $O/fullsize.log
# A/B of config 4 (5 steps each): the default, 32 waves/CU (64 VGPRs with spills), 2 scans, u32 counters
ab() { timeout -k 10 200 env "$@" python bench.py --config c4 --steps 5 --warmup 2 --no-cpu > $O/ab.log 2>&1 || { echo AB_FAIL "$@"; tail -5 $O/ab.log; return 1; }
  grep '^{' $O/ab.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$*', round(d['value']/1e9,3), 'Gtr/s', round(d['roofline']['kernel_ms'],3), 'ms', d['config']['launch']['wg_threads'], d['config']['launch']['blocks_per_cu'])"; }
ab X=0 && ab ISIM_LIB=istio-isotope_amd/isim/libisim_wpe8.so ISIM_TREE_THREADS=1024 && ab ISIM_LIB=istio-isotope_amd/isim/libisim_scan2.so && ab ISIM_TREE_CNT32=1 || exit 10
bash tools/profile_cfg.sh c4 "--config c4 --no-cpu" > $O/prof_c4.log 2>&1 || { echo PROF_C4_FAIL; tail -5 $O/prof_c4.log; exit 8; }
bash tools/profile_cfg.sh c3p "--config c3p --no-cpu --no-wave-leg" > $O/prof_c3p.log 2>&1 || { echo PROF_C3P_FAIL; tail -5 $O/prof_c3p.log; exit 7; }
echo prof done
