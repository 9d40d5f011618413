#!/bin/bash
# Round 4: decapsulate into line-aligned slots (align 0): the strided text-grid open vs
# the descriptor kernels + scatter (WG_TUNN_STRIDED 1 / 0), interleaved; plus the
# rocprofv3 kernel trace of one of each.  usage: tools/gpu_r04_strided.sh TAG
set -euo pipefail
TAG=${1:-r04st}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG}_strided.jsonl
: > $OUT
for rep in 1 2 3; do
  for s in 1 0; do
    timeout -k 10 180 env WG_TUNN_STRIDED=$s python tools/bench_tunn.py --sizes 262144 --reps 7 --register --align 0 >> $OUT
  done
done
for s in 1 0; do
  timeout -k 10 120 env WG_TUNN_STRIDED=$s rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/${TAG}_trace_s$s -o run -- python tools/bench_tunn.py --sizes 262144 --reps 3 --register --align 0 \
    > gpurun_out/${TAG}_trace_s$s.log 2>&1
  python tools/tunn_timeline.py gpurun_out/${TAG}_trace_s$s > gpurun_out/${TAG}_timeline_s$s.jsonl
done
