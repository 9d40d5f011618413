#!/bin/bash
# Round 4: the auto output mode (direct where the output runs sit on whole lines, else
# scatter) at destination alignments 0 / 16 / 64 past a page, after the Tunn GPU tests;
# then 5 runs at numpy's own placement.  usage: tools/gpu_r04_align2.sh TAG
set -euo pipefail
TAG=${1:-r04al2}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_align.jsonl
: > $OUT
for rep in 1 2 3; do
  for al in 0 16 64; do
    timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --register --align $al >> $OUT
  done
done
for rep in 1 2 3 4 5; do
  timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --register >> $OUT
done
