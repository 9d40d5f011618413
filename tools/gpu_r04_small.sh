#!/bin/bash
# Round 4: per-call cost of small Tunn batches (the gateway's regime; NepTUN's default
# batch is 50 packets): bench_tunn at 64 .. 16384 packets, phases per call, for the pool's
# spin (WG_TUNN_SPIN_US 20 vs 0) and the staged path's zero-copy vs explicit copies; the
# Tunn GPU tests first.  usage: tools/gpu_r04_small.sh TAG
set -euo pipefail
TAG=${1:-r04sm}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
OUT=gpurun_out/${TAG}_small.jsonl
: > $OUT
for envs in "WG_TUNN_SPIN_US=20" "WG_TUNN_SPIN_US=0" "WG_TUNN_SPIN_US=20 WG_TUNN_ZEROCOPY=0"; do
  timeout -k 10 300 env $envs python tools/bench_tunn.py --sizes 64,256,1024,4096,16384 --reps 30 --phase-timing >> $OUT
  timeout -k 10 300 env $envs python tools/bench_tunn.py --sizes 64,256,1024,4096,16384 --reps 30 --phase-timing --register >> $OUT
done
timeout -k 10 300 python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
