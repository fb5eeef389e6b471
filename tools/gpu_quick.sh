set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 tools/philox_peak.hip -o gpurun_out/pp 2>/dev/null || exit 10
timeout -k 10 120 gpurun_out/pp > gpurun_out/philox_peak.json || exit 11
cat gpurun_out/philox_peak.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_walk_gpu.py -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 12; }
tail -1 gpurun_out/t.log
for a in "--config c3" "--config c3 --mode B" "--config c4 --batch 1048576"; do
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $a > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().split(chr(10))[-1]);print('$a', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', d.get('compute_roofline') and round(d['compute_roofline']['frac'],3))"
done
