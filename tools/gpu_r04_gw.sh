#!/bin/bash
# Round 4: the UDP gateway example with its packet pools registered (DMA path) vs plain
# malloc'd pools -- the gateway GPU test in both forms, then tools/bench_gateway.py
# (262,144 x 1350 B, batches 1024 / 4096 / 16384, 1 / 4 / 8 peers).
# usage: tools/gpu_r04_gw.sh TAG
set -euo pipefail
TAG=${1:-r04y}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_udp_gateway.py \
  > gpurun_out/${TAG}_pytest_gw.txt 2>&1
GW_PAIRS="1 4 8" GW_REG="0 1" timeout -k 10 900 python tools/bench_gateway.py 262144 1350 1024 4096 16384 \
  > gpurun_out/${TAG}_gateway.jsonl 2> gpurun_out/${TAG}_gateway.err
