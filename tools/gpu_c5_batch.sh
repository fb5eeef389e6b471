set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in ${BATCHES:-65536 131072 262144}; do
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu --batch $b > gpurun_out/c5_$b.log 2>&1 || { tail -5 gpurun_out/c5_$b.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/c5_$b.log').read().strip().split(chr(10))[-1]);print($b, round(d['value']/1e6,3), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms', round(d['roofline']['frac'],3), d['config']['des_rows'], d['mean_latency_ns'])"
done
