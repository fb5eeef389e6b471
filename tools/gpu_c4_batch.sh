set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in 16777216 33554432 67108864; do
timeout -k 10 300 python bench.py --config c4 --no-cpu --steps 5 --warmup 2 --batch $b > gpurun_out/c4b.log 2>&1 || { tail -5 gpurun_out/c4b.log; exit 13; }
grep '^{' gpurun_out/c4b.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print($b, round(d['value']/1e6,2),'Mtr/s', round(d['ms_per_step'],3),'ms/step')"
done
