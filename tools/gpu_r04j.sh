#!/bin/bash
# Round 4: timeline of the registered (DMA) Tunn path -- rocprofv3 kernel + memory-copy trace
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r04j_trace -o run -- \
  python tools/bench_tunn.py --sizes 262144 --reps 3 --register > gpurun_out/r04j_trace.log 2>&1
