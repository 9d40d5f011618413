#!/bin/bash
# Round 4: batched Tunn host path -- GPU tests, then tools/bench_tunn.py at 262,144 x
# 1350 B in several data-movement modes (interleaved, twice), with per-phase host /
# device times; optionally the pinned pipe (tools/bench_e2e.py) on the same box.
# usage: tools/gpu_r04_tunn.sh TAG [full] [e2e]   (outputs gpurun_out/TAG_*)
set -euo pipefail
TAG=${1:-r04t}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
if [ "${2:-}" = "full" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tunn_gpu.py \
    > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
fi
OUT=gpurun_out/${TAG}_tunn.jsonl
: > $OUT
run() {  # "ENV=.. ENV=.." [--register]
  local envs=$1; shift
  timeout -k 10 180 env $envs python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing "$@" >> $OUT
}
for rep in 1 2; do
  run "WG_TUNN_ZEROCOPY=1 WG_TUNN_NT=1"
  run "WG_TUNN_ZEROCOPY=1 WG_TUNN_NT=1 WG_TUNN_CHUNK_KB=65536"
  run "WG_TUNN_DMA=1" --register
  run "WG_TUNN_DMA=1 WG_TUNN_SETS=3" --register
  run "WG_TUNN_DMA=1 WG_TUNN_CHUNK_KB=65536" --register
  run "WG_TUNN_DMA=1 WG_TUNN_CHUNK_KB=65536 WG_TUNN_SETS=3" --register
  run "WG_TUNN_DMA=1 WG_TUNN_CHUNK_KB=32768 WG_TUNN_SETS=4" --register
  run "WG_TUNN_DMA=0" --register
done
if [ "${3:-}" = "e2e" ]; then
  timeout -k 10 300 python tools/bench_e2e.py > gpurun_out/${TAG}_e2e.jsonl 2> gpurun_out/${TAG}_e2e.err
fi
