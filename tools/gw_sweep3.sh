#!/bin/bash
# the gateway sweep three times over (cells move by +-20 % run to run): GPU plain /
# registered and the CPU line, batch 1024 / 4096 / 16384 x 1 / 2 / 4 / 8 peers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r05w}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2 3; do
  GW_ARGS="262144 1350 1024 4096 16384" GW_PAIRS="1 2 4 8" GW_REG="0 1" GW_MUX="0" GW_BACKEND="gpu cpu" \
    tools/gpu.sh $TAG gateway > /dev/null || exit 1
  cat $OUT/gateway.jsonl >> $OUT/sweep3.jsonl
done
wc -l $OUT/sweep3.jsonl
