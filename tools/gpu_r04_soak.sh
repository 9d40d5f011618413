#!/bin/bash
# Round 4: randomized soak of the batched Tunn's registered-pool paths against the model
# (tests/soak_tunn.py), two seeds.  usage: tools/gpu_r04_soak.sh TAG SECONDS
set -euo pipefail
TAG=${1:-r04soak}
S=${2:-240}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 $((S + 120)) python -u tests/soak_tunn.py $S 1 > gpurun_out/${TAG}_seed1.jsonl 2> gpurun_out/${TAG}_seed1.err
timeout -k 10 $((S + 120)) python -u tests/soak_tunn.py $S 2 > gpurun_out/${TAG}_seed2.jsonl 2> gpurun_out/${TAG}_seed2.err
