#!/bin/bash
# Round 3 (h): the affine descriptor groups -- GPU suite on the product build,
# descriptor A/B (base = WG_DESC_AFFINE=0, aff = product, affsd = + shared first
# diagonal round), then the config-4 bench line.  gpurun_out/r03h/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CHECK_DESC="base aff affsd" bash tools/gpu_r03_check.sh r03h || exit $?
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03h/bench_config4.json 2> gpurun_out/r03h/bench_config4.err || exit $?
tail -c 1500 gpurun_out/r03h/bench_config4.json
