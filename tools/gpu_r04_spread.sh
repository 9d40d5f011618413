#!/bin/bash
# Round 4: spread launches for under-filled grids (WG_SPREAD) and the last round's
# single keystream block (WG_LAST_ONE_BLOCK) -- the GPU suite on the default build,
# then same-process A/Bs of the def / spread0 / lob0 variant builds (tools/ab.py:
# bit-identical output required, interleaved rounds) on under-filled shapes (8 KiB at
# the bench's step payload, Tunn-chunk-sized batches, config 4 with few packets), the
# one-block size (192 B) and the full-size configs 2 / 3 / 4.
# usage: tools/gpu_r04_spread.sh TAG   (outputs gpurun_out/TAG_*)
set -euo pipefail
TAG=${1:-r04n}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest_gpu.txt 2>&1
V=build/variants
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
ab() {  # "ENV=.. ENV=.."
  echo "== $1" >> $OUT
  timeout -k 10 300 env $1 python tools/ab.py $V/libneptun_gpu_def.so $V/libneptun_gpu_spread0.so \
    $V/libneptun_gpu_lob0.so >> $OUT 2>&1
}
ab "AB_SIZE=8192 AB_N=172544"
ab "AB_SIZE=1350 AB_N=12288"
ab "AB_SIZE=1350 AB_N=131072"
ab "AB_SIZE=192 AB_N=7372800"
ab "AB_SIZE=128 AB_N=4194304"
ab "AB_SIZE=1350"
ab "AB_CONFIG=4 AB_PEERS=64 AB_PER_PEER=256"
ab "AB_CONFIG=4"
ab "AB_CONFIG=3"
