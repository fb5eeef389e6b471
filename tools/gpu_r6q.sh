#!/bin/bash
# round 6: where c3p's / c3s's WRITE goes — WRITE_SIZE per launch with and
# without records / duration rows, and with the sinks compiled out (TREE_NO_SINK)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c3p c3s; do
  for f in "" "--no-records" "--no-svc-dur" "--no-records_--no-svc-dur"; do
    echo "== $c ${f//_/ }"
    LIBS="libisim.so libisim_nosink.so" CFG="--config $c ${f//_/ }" PMC="WRITE_SIZE" timeout -k 10 300 bash tools/gpu_pmc_ab.sh 2>&1 | grep -v "pmcab done" || exit 7
  done
done
