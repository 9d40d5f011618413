#!/bin/bash
# Round 4: registered (DMA) Tunn path, chunk size x staging sets, with pack sub-phases.
# usage: tools/gpu_r04_tunn2.sh TAG
set -euo pipefail
TAG=${1:-r04t2}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG}_tunn.jsonl
: > $OUT
run() { local envs=$1; shift; timeout -k 10 180 env $envs python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing "$@" >> $OUT; }
for rep in 1 2; do
  run "WG_TUNN_CHUNK_KB=16384 WG_TUNN_SETS=3" --register
  run "WG_TUNN_CHUNK_KB=32768 WG_TUNN_SETS=3" --register
  run "WG_TUNN_CHUNK_KB=65536 WG_TUNN_SETS=3" --register
  run "WG_TUNN_CHUNK_KB=65536 WG_TUNN_SETS=4" --register
  run "WG_TUNN_CHUNK_KB=131072 WG_TUNN_SETS=3" --register
done
