#!/bin/bash
# walk parity (every walk test file) + A/B on c3 + WRITE_SIZE of both libraries
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/stage
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_walk_gpu.py tests/test_fullsize_gpu.py tests/test_kat_gpu.py tests/test_golden_records_gpu.py tests/test_multi_gpu.py -m gpu > gpurun_out/stage/t.log 2>&1 || { tail -30 gpurun_out/stage/t.log; exit 12; }
tail -1 gpurun_out/stage/t.log
REPS=2 LIBS="libisim_base.so libisim.so" CONFIGS="--config c3 --no-mode-b;--config c3 --mode B --no-mode-b" bash tools/ab_libs.sh || exit 13
cd /tmp && export TMPDIR=/tmp
for lib in libisim_base.so libisim.so; do
ISIM_LIB=$GRAFT_REPO_ROOT/istio-isotope_amd/isim/$lib timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/stage/w_$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --no-mode-b --steps 2 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/stage/w_$lib.log 2>&1 || exit 14
python3 -c "
import csv,glob
f=glob.glob('$GRAFT_REPO_ROOT/gpurun_out/stage/w_$lib/**/*counter_collection.csv',recursive=True)[0]
v=[float(r['Counter_Value']) for r in csv.DictReader(open(f)) if 'isim_walk' in r['Kernel_Name'] and r['Counter_Name']=='WRITE_SIZE']
print('$lib WRITE_SIZE KB per launch', sum(v)/len(v))"
done
