#!/bin/bash
# round 6: the cdag bench batch, then the bench lines (c3 with its mode-B
# legs, c3p, c3s, c4w, cdag, c4), then LDS-conflict A/B of kind 7 on config 4
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6b
O=gpurun_out/r6b
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  "tests/test_fullsize_gpu.py::test_cdag_bench_batch" > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for c in c3 c3p c3s c4w cdag c4; do
timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 6; }
grep '^{' $O/bench_$c.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c', d['value'], d['roofline']['kernel_ms'], {k:(d[k]['value'],d[k]['kernel_ms'],d[k]['kernel_kind']) for k in ('mode_b','mode_b_informative') if k in d}, d.get('speedup_vs_wave_walk'))"
done
LIBS="libisim.so libisim_nohist.so libisim_nosink.so" CFG="--config c4" \
  PMC="SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
  timeout -k 10 600 bash tools/gpu_pmc_ab.sh 2>&1 | tail -5
echo r6b done
