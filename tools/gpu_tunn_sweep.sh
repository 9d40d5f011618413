#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tunn
for zc in 0 1; do for ck in 4096 16384 65536; do
  echo "zerocopy=$zc chunk_kb=$ck"
  WG_TUNN_ZEROCOPY=$zc WG_TUNN_CHUNK_KB=$ck timeout -k 10 120 python tools/bench_tunn.py --sizes 16384,65536 --reps 7 2>>gpurun_out/tunn/sweep.err || exit 1
done; done
