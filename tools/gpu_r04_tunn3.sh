#!/bin/bash
# Round 4: the batched Tunn's final host-path numbers -- 5 runs each of the registered
# (DMA batch) and the staged (unregistered buffers) paths at 262,144 x 1350 B, plus
# 65,536 and 1,048,576-packet batches once.  usage: tools/gpu_r04_tunn3.sh TAG [ENV...]
set -euo pipefail
TAG=${1:-r04t3}
shift || true
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG}_tunn.jsonl
: > $OUT
for rep in 1 2 3 4 5; do
  timeout -k 10 180 env "$@" python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
  timeout -k 10 180 env "$@" python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing >> $OUT
done
timeout -k 10 300 env "$@" python tools/bench_tunn.py --sizes 65536,1048576 --reps 5 --phase-timing --register >> $OUT
