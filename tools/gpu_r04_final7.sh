#!/bin/bash
# Round 4: final batched Tunn runs with 4 staging sets for DMA batches -- the Tunn GPU
# tests, 5 runs at numpy's placement, 5 with page-aligned pools, 64 Ki / 1M once.
# usage: tools/gpu_r04_final7.sh TAG
set -euo pipefail
TAG=${1:-r04f7}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_tunn.jsonl
: > $OUT
for rep in 1 2 3 4 5; do
  timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
  timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register --align 0 >> $OUT
done
timeout -k 10 300 python tools/bench_tunn.py --sizes 65536,1048576 --reps 5 --phase-timing --register >> $OUT
