#!/bin/bash
# Round 3 (l): text-grid load policies split by piece kind (WG_TEXT_SPLIT): the
# head piece (next line's first 16 B, read again next round) vs the body pieces
# (this line's last access).  Timing A/B on NepTUN's offset-0 open + PMC traffic
# per variant.  gpurun_out/r03l/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03l
mkdir -p $OUT
V=build/variants
LIBS="$V/libneptun_gpu_base.so $V/libneptun_gpu_tsplit.so $V/libneptun_gpu_tsplitrev.so $V/libneptun_gpu_tsplit00.so"
timeout -k 10 300 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $LIBS > $OUT/ab_text.log 2>&1 || { tail -20 $OUT/ab_text.log; exit 1; }
grep -v amdgpu.ids $OUT/ab_text.log | tail -8
timeout -k 10 500 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 python tools/pmc_ab.py $OUT/pmc_text.json $LIBS > $OUT/pmc_text.log 2>&1 || { tail -20 $OUT/pmc_text.log; exit 1; }
grep -v amdgpu.ids $OUT/pmc_text.log | tail -8
