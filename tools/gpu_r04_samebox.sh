#!/bin/bash
# Round 4: the pinned host pipe (tools/bench_e2e.py) and the registered batched Tunn on
# the same box, interleaved, so the Tunn's fraction of the link is read off one machine.
# usage: tools/gpu_r04_samebox.sh TAG
set -euo pipefail
TAG=${1:-r04sb}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG}_tunn.jsonl
: > $OUT
for rep in 1 2 3; do
  timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
done
timeout -k 10 400 python tools/bench_e2e.py > gpurun_out/${TAG}_e2e.jsonl 2> gpurun_out/${TAG}_e2e.err
for rep in 1 2; do
  timeout -k 10 180 python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register >> $OUT
done
