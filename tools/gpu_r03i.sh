#!/bin/bash
# Round 3 (i): affine descriptor kernel as its own kernel (unordered launches) --
# GPU suite, descriptor A/B (base = WG_DESC_AFFINE=0, aff = product, affsd = +
# shared first diagonal round), open-grid A/B on NepTUN's offset-0 open (text
# grid = product vs the wire grid with straddling output lines, nt / default
# stores), then the config-4 profile (bench line, trace, PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CHECK_DESC="base aff affsd" bash tools/gpu_r03_check.sh r03i || exit $?
V=build/variants
timeout -k 10 300 env AB_PAD=0 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_aff.so $V/libneptun_gpu_wgrid.so $V/libneptun_gpu_wgriddef.so > gpurun_out/r03i/open_grid.log 2>&1 || { tail -20 gpurun_out/r03i/open_grid.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03i/open_grid.log | tail -8
bash tools/gpu_profile.sh r03i_prof 4
