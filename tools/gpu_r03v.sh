#!/bin/bash
# Round 3 (v): XCD-contiguous persistent walk (WG_XCD_CONTIG) vs the product's
# round-robin walk, config 2 (wire grid + padding) and NepTUN's offset-0 open.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03v
mkdir -p $OUT
V=build/variants
timeout -k 10 300 env AB_PAD=1 AB_BURST=100 AB_ROUNDS=7 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_xcd.so > $OUT/ab_wire.log 2>&1 || { tail -20 $OUT/ab_wire.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_wire.log | tail -4
timeout -k 10 300 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=7 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_xcd.so > $OUT/ab_text.log 2>&1 || { tail -20 $OUT/ab_text.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_text.log | tail -4
