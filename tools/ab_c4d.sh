set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "" ISIM_DES_ITEMS_FAT_QUIET "" ISIM_DES_ITEMS_FAT_QUIET; do
  if [ -n "$v" ]; then export $v=1; else unset ISIM_DES_ITEMS_FAT_QUIET; fi
  ISIM_DES_DEBUG=1 timeout -k 10 300 python -u bench.py --config c4d --steps 3 --warmup 1 --no-cpu > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "$v $(grep '^{' gpurun_out/ab.log | python -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])') $(grep passes gpurun_out/ab.log | tail -1)"
done
