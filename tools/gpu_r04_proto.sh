#!/bin/bash
# Round 4: copy-engine microbenchmark + the K-lanes-per-packet seal prototype
# (tools/proto_xlane.hip): bit-exact check, A/B timing.   usage: tools/gpu_r04_proto.sh TAG
set -euo pipefail
TAG=${1:-r04p}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 build/proto/microbench_dma 1350 > gpurun_out/${TAG}_dma.jsonl
timeout -k 10 120 build/proto/microbench_dma 1408 >> gpurun_out/${TAG}_dma.jsonl
for P in 1350 8192; do
  timeout -k 10 180 python tools/proto_xlane.py check --size $P >> gpurun_out/${TAG}_xlane_check.jsonl
done
for P in 1350 8192; do
  timeout -k 10 240 python tools/proto_xlane.py ab --size $P --rounds 11 --burst 30 >> gpurun_out/${TAG}_xlane_ab.jsonl
done
