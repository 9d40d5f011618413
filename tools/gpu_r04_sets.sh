#!/bin/bash
# Round 4: staging sets (WG_TUNN_SETS 2 / 3 / 4) for the DMA batches' scatter chunks --
# decapsulate into line-aligned slots (align 0) and encapsulate at numpy's placement.
# usage: tools/gpu_r04_sets.sh TAG
set -euo pipefail
TAG=${1:-r04se}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG}_sets.jsonl
: > $OUT
for rep in 1 2; do
  for al in 0 16; do
    for sets in 2 3 4; do
      timeout -k 10 180 env WG_TUNN_SETS=$sets python tools/bench_tunn.py --sizes 262144 --reps 7 --register --align $al >> $OUT
    done
  done
done
