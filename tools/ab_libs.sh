# A/B of libisim builds on the GPU box: bench.py per library and workload
# (build the variants in-tree first, e.g. libisim_base.so from a stash).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
LIBS=${LIBS:-"libisim_base.so libisim.so"}
for rep in $(seq ${REPS:-2}); do
for lib in $LIBS; do
IFS=';' read -ra CFGS <<< "${CONFIGS:---config c3;--config c3 --mode B;--config c4;--config c2}"
for a in "${CFGS[@]}"; do
ISIM_LIB=$PWD/istio-isotope_amd/isim/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu $a > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 13; }
python -c "import json;d=json.loads(open('gpurun_out/b.log').read().strip().split(chr(10))[-1]);print('$lib $a', round(d['value']/1e6,2), 'Mtr/s', round(d['roofline']['kernel_ms'],3), 'ms')"
done; done; done
