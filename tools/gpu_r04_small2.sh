#!/bin/bash
# Round 4: small-batch GPU round trip -- polling the chunk events (WG_TUNN_POLL_US 50 vs 0)
# and one stream per DMA chunk (WG_TUNN_DMA_STREAMS=0), bench_tunn at 64 .. 16384 packets;
# the Tunn GPU tests first.  usage: tools/gpu_r04_small2.sh TAG
set -euo pipefail
TAG=${1:-r04sm3}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_small.jsonl
: > $OUT
for envs in "WG_TUNN_POLL_US=50" "WG_TUNN_POLL_US=0" "WG_TUNN_POLL_US=50 WG_TUNN_DMA_STREAMS=0"; do
  timeout -k 10 300 env $envs python tools/bench_tunn.py --sizes 64,256,1024,4096,16384 --reps 30 --phase-timing >> $OUT
  timeout -k 10 300 env $envs python tools/bench_tunn.py --sizes 64,256,1024,4096,16384 --reps 30 --phase-timing --register >> $OUT
done
timeout -k 10 300 python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
