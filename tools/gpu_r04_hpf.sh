#!/bin/bash
# Round 4: open's header prefetch (WG_OPEN_HDR_PREFETCH=1, variant hpf1) against the
# product (def) at the small packet sizes, where open runs ~45 % behind seal
# (r04n), and at 1350 B on both open grids.  usage: tools/gpu_r04_hpf.sh TAG
set -euo pipefail
TAG=${1:-r04o}
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
V=build/variants
OUT=gpurun_out/${TAG}_ab_hpf.txt
: > $OUT
ab() {
  echo "== $1" >> $OUT
  timeout -k 10 300 env $1 python tools/ab.py $V/libneptun_gpu_def.so $V/libneptun_gpu_hpf1.so >> $OUT 2>&1
}
ab "AB_SIZE=128 AB_N=4194304"
ab "AB_SIZE=192 AB_N=4194304"
ab "AB_SIZE=576 AB_N=2097152"
ab "AB_SIZE=1350"
ab "AB_SIZE=128 AB_N=4194304 AB_OPEN_OFF=0"
