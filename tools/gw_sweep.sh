#!/bin/bash
# concurrent-caller probe + the gateway sweep (GPU: plain, registered, mux; CPU line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r05j}
OUT=gpurun_out/$TAG; mkdir -p $OUT
gcc -O2 -pthread -Iinclude -DTT_ENGINES tools/tunn_threads.c -Lneptun_amd -lneptun_gpu -Wl,-rpath,$PWD/neptun_amd -o /tmp/tt5 || exit 1
for T in 1 4 8; do
  for v in "/tmp/tt5" "GW_PRIVATE_ENGINES=1 /tmp/tt5"; do
    timeout -k 10 120 env $v $T 4096 48 | sed "s#^{#{\"variant\": \"$v\", #" >> $OUT/tt.jsonl || exit 1
  done
done
cut -c1-200 $OUT/tt.jsonl
GW_ARGS="262144 1350 1024 4096 16384" GW_PAIRS="1 2 4 8" GW_REG="0 1" GW_MUX="0 1" GW_BACKEND="gpu cpu" \
  tools/gpu.sh $TAG gateway
