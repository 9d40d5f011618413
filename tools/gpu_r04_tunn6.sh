#!/bin/bash
# Round 4: DMA batches' chunk ramp (WG_TUNN_RAMP=1 default vs 0), interleaved, then the
# final 5-run numbers (tools/gpu_r04_tunn3.sh) -- after the Tunn GPU tests.
# usage: tools/gpu_r04_tunn6.sh TAG
set -euo pipefail
TAG=${1:-r04u}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_ramp.jsonl
: > $OUT
for rep in 1 2 3; do
  for envs in "WG_TUNN_RAMP=1" "WG_TUNN_RAMP=0" "WG_TUNN_RAMP=1 WG_TUNN_CHUNK_KB=32768"; do
    timeout -k 10 180 env $envs python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
  done
done
bash tools/gpu_r04_tunn3.sh ${TAG}
