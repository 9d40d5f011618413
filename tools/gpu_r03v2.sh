#!/bin/bash
# Round 3 (v2): XCD-contiguous walk confirmation -- both orders, 11 rounds, config 2 bench layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03v
mkdir -p $OUT
V=build/variants
timeout -k 10 300 env AB_PAD=1 AB_BURST=100 AB_ROUNDS=25 python tools/ab.py $V/libneptun_gpu_xcd.so $V/libneptun_gpu_base.so > $OUT/ab_wire_rev.log 2>&1 || { tail -20 $OUT/ab_wire_rev.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_wire_rev.log | tail -2
timeout -k 10 300 env AB_PAD=1 AB_BURST=100 AB_ROUNDS=25 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_xcd.so > $OUT/ab_wire_fwd.log 2>&1 || { tail -20 $OUT/ab_wire_fwd.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_wire_fwd.log | tail -2
timeout -k 10 400 env AB_CONFIG=4 AB_PER_PEER=1024 AB_BURST=6 AB_ROUNDS=8 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_xcd.so > $OUT/ab_config4.log 2>&1 || { tail -20 $OUT/ab_config4.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_config4.log | tail -2
