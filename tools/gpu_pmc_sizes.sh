#!/bin/bash
# HBM traffic of the descriptor kernels per payload size (config 3's sizes one at a
# time, tools/pmc_traffic.py): where config 3's traffic above the algorithmic bytes
# comes from.  Outputs gpurun_out/$TAG/pmc_traffic_size<P>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for spec in 64:1048576 256:1048576 576:524288 1350:262144 8900:65536; do
  P=${spec%%:*}; N=${spec##*:}
  echo "== size $P x $N"
  timeout -k 10 300 python tools/pmc_traffic.py "$OUT/pmc_traffic_size$P.json" --config 3 --mixed-sizes $P --per-size $N \
    > "$OUT/pmc_size$P.log" 2>&1 || { echo "size $P failed"; tail -5 "$OUT/pmc_size$P.log"; exit 1; }
done
echo "== done"
