#!/bin/bash
# Round 3 (q): occupancy 3 (384-thread workgroups, 2 per CU, 168-VGPR cap) against
# the product's occupancy 4 (512-thread workgroups) on config 2 -- wire grid with slot
# padding (the bench) and NepTUN's offset-0 open (text grid).  gpurun_out/r03q/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03q
mkdir -p $OUT
V=build/variants
timeout -k 10 300 env AB_PAD=1 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_occ3.so > $OUT/ab_wire.log 2>&1 || { tail -20 $OUT/ab_wire.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_wire.log | tail -4
timeout -k 10 300 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_base.so $V/libneptun_gpu_occ3.so > $OUT/ab_text.log 2>&1 || { tail -20 $OUT/ab_text.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_text.log | tail -4
