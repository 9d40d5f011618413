#!/bin/bash
# Round 4: the DMA batches' scatter output with the copy / kernel / output streams split
# and the scatter grid capped (WG_TUNN_SCATTER_BLOCKS) vs one stream per set and a full
# grid (the previous form), at destination alignments 0 and 16; the Tunn GPU tests first.
# usage: tools/gpu_r04_scatter.sh TAG
set -euo pipefail
TAG=${1:-r04sc}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_scatter.jsonl
: > $OUT
for rep in 1 2; do
  for al in 0 16; do
    for envs in "WG_TUNN_DMA_STREAMS=1" "WG_TUNN_DMA_STREAMS=0 WG_TUNN_SCATTER_BLOCKS=0" \
                "WG_TUNN_DMA_STREAMS=1 WG_TUNN_SCATTER_BLOCKS=0" "WG_TUNN_DMA_STREAMS=1 WG_TUNN_SCATTER_BLOCKS=128"; do
      timeout -k 10 180 env $envs python tools/bench_tunn.py --sizes 262144 --reps 7 --register --align $al >> $OUT
    done
  done
done
