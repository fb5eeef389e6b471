#!/bin/bash
# One SQ instruction-count PMC pass per libisim build on a bench config:
#   LIBS="libisim_base.so libisim.so" CFG="--config c4" bash tools/gpu_pmc_ab.sh
# An entry may carry environment settings: "libisim.so:ISIM_DES_TREELET=0,X=1"
# (KNAME: the kernel-name filter, default isim_tree).
# Output: gpurun_out/pmcab/<entry>/ (rocprofv3 csv) + a one-line summary per entry.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ent in ${LIBS:-libisim_base.so libisim.so}; do
  IFS=: read lib envs <<< "$ent"
  lib=${lib}; tag=${ent//[:=,]/_}
  [ -n "$envs" ] && export ${envs//,/ }
  ISIM_LIB=$R/istio-isotope_amd/isim/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES} -d $O/$tag -o run --output-format csv -- python3 $R/bench.py ${CFG:---config c4} --steps 2 --warmup 1 --no-cpu > $O/$tag.log 2>&1 || { echo "$tag pmc failed"; tail -5 $O/$tag.log; exit 12; }
  python3 - "$O/$tag" "$tag" "${KNAME:-isim_tree}" <<'PY'
import csv, glob, sys, collections
d, lib, kn = sys.argv[1:4]
rows = []
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(float); disp = set()
for r in rows:
    if kn not in r.get("Kernel_Name", ""): continue
    disp.add(r["Dispatch_Id"]); agg[r["Counter_Name"]] += float(r["Counter_Value"])
n = max(1, len(disp))
print(lib, "dispatches", n, " ".join(f"{k}={v/n:.4g}" for k, v in sorted(agg.items())))
PY
  [ -n "$envs" ] && for e in ${envs//,/ }; do unset ${e%%=*}; done
done
echo pmcab done
