#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/diag2
mkdir -p $OUT
timeout -k 10 120 ./tools/microbench_mem2 > $OUT/mem2.txt 2>&1; cat $OUT/mem2.txt
./tools/pmc.sh $OUT/pmc_v1 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
