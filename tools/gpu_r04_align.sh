#!/bin/bash
# Round 4: DMA batches' output mode vs the destination slots' alignment: slot 0 at 0 or 16
# bytes past a page (the seal's datagram / the open's wire grid on whole 128-byte lines, or
# not), WG_TUNN_DMA_OUT direct vs scatter, 262,144 x 1350 B registered, interleaved twice.
# usage: tools/gpu_r04_align.sh TAG
set -euo pipefail
TAG=${1:-r04al}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG}_align.jsonl
: > $OUT
for rep in 1 2; do
  for al in 0 16 64; do
    for o in direct scatter; do
      timeout -k 10 180 env WG_TUNN_DMA_OUT=$o python tools/bench_tunn.py --sizes 262144 --reps 7 --register \
        --align $al >> $OUT
    done
  done
done
timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --register >> $OUT
