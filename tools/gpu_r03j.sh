#!/bin/bash
# Round 3 (j): descriptor kernels by launch kind -- affine groups (unordered
# launches) and the SGPR-key forms of single-slot contexts.  GPU suite on the
# product, descriptor A/B on configs 4 and 3 (base = neither, aff = affine only,
# key1 = product, affsd = product + shared first diagonal round for per-lane
# keys), open-grid A/B on NepTUN's offset-0 open (text grid = product vs the
# wire grid with straddling output lines, nt / default stores), then the
# config 3 / 4 profile (bench lines, traces, PMC).  gpurun_out/r03j*/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CHECK_DESC="base aff key1 affsd" bash tools/gpu_r03_check.sh r03j || exit $?
V=build/variants
timeout -k 10 300 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_key1.so $V/libneptun_gpu_wgrid.so $V/libneptun_gpu_wgriddef.so > gpurun_out/r03j/open_grid.log 2>&1 || { tail -20 gpurun_out/r03j/open_grid.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03j/open_grid.log | tail -8
bash tools/gpu_profile.sh r03j_prof 3 4
