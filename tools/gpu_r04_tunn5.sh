#!/bin/bash
# Round 4: the batched Tunn's final numbers on the default build -- the Tunn GPU tests,
# then tools/gpu_r04_tunn3.sh (5 runs each of the registered and the staged paths at
# 262,144 x 1350 B, plus 65,536 / 1,048,576-packet registered batches).
# usage: tools/gpu_r04_tunn5.sh TAG
set -euo pipefail
TAG=${1:-r04t}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_tunn_gpu.py \
  > gpurun_out/${TAG}_pytest_tunn.txt 2>&1
bash tools/gpu_r04_tunn3.sh ${TAG}
