#!/bin/bash
# Round 4: DMA batches with direct output (the AEAD kernel writes the caller's dst)
# vs staged output + scatter kernel (WG_TUNN_DMA_OUT=scatter), on separate copy /
# kernel streams or all on the staging set's stream (WG_TUNN_DMA_STREAMS=0): the Tunn
# GPU tests, bench_tunn at 262,144 x 1350 B interleaved, one rocprofv3 kernel +
# memory-copy trace per output form (tools/tunn_timeline.py).
# usage: tools/gpu_r04_tunn4.sh TAG   (outputs gpurun_out/TAG_*)
set -euo pipefail
TAG=${1:-r04q}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_tunn.jsonl
: > $OUT
for rep in 1 2 3; do
  for envs in "WG_TUNN_DMA_OUT=direct" "WG_TUNN_DMA_OUT=scatter WG_TUNN_DMA_STREAMS=0" \
              "WG_TUNN_DMA_OUT=direct WG_TUNN_CHUNK_KB=32768" "WG_TUNN_DMA_OUT=direct WG_TUNN_CHUNK_KB=8192" \
              "WG_TUNN_DMA_OUT=direct WG_TUNN_SETS=2" "WG_TUNN_DMA_OUT=direct WG_TUNN_DMA_STREAMS=0"; do
    timeout -k 10 180 env $envs python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
  done
done
for o in direct scatter; do
  timeout -k 10 120 env WG_TUNN_DMA_OUT=$o rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/${TAG}_trace_$o -o run -- python tools/bench_tunn.py --sizes 262144 --reps 3 --register \
    > gpurun_out/${TAG}_trace_$o.log 2>&1
  python tools/tunn_timeline.py gpurun_out/${TAG}_trace_$o > gpurun_out/${TAG}_timeline_$o.jsonl
done
