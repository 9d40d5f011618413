#!/bin/bash
# Round 3 (y): open header prefetch (WG_OPEN_HDR_PREFETCH) -- the GPU suite on the
# variant (in this box's scratch copy), then A/B against the product build on config 2
# (wire grid + padding, both orders, 25 rounds) and NepTUN's offset-0 open.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03y
mkdir -p $OUT
V=build/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "every_group or full_size or randomized" --timeout 120 --timeout-method thread > $OUT/pytest_product.log 2>&1 || { tail -20 $OUT/pytest_product.log; exit 1; }
tail -1 $OUT/pytest_product.log
cp neptun_amd/libneptun_gpu.so $OUT/product.so.bak && cp $V/libneptun_gpu_hpf.so neptun_amd/libneptun_gpu.so || exit 1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_hpf.log 2>&1 || { tail -20 $OUT/pytest_hpf.log; exit 1; }
tail -1 $OUT/pytest_hpf.log
cp $OUT/product.so.bak neptun_amd/libneptun_gpu.so && rm -f $OUT/product.so.bak || exit 1
timeout -k 10 300 env AB_PAD=1 AB_BURST=100 AB_ROUNDS=25 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_hpf.so > $OUT/ab_fwd.log 2>&1 || { tail -20 $OUT/ab_fwd.log; exit 1; }
grep med $OUT/ab_fwd.log
timeout -k 10 300 env AB_PAD=1 AB_BURST=100 AB_ROUNDS=25 python tools/ab.py $V/libneptun_gpu_hpf.so $V/libneptun_gpu_base.so > $OUT/ab_rev.log 2>&1 || { tail -20 $OUT/ab_rev.log; exit 1; }
grep med $OUT/ab_rev.log
timeout -k 10 300 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=11 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_hpf.so > $OUT/ab_text.log 2>&1 || { tail -20 $OUT/ab_text.log; exit 1; }
grep med $OUT/ab_text.log
