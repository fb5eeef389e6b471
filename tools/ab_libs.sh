set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in libisim.so libisim_w6.so libisim_w7.so; do
for a in "--config c3" "--config c3 --mode B"; do
ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $a > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().split(chr(10))[-1]);print('$lib $a', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms')"
done; done
