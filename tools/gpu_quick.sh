#!/bin/bash
# Quick GPU iteration: parity tests, then bench (no CPU baseline), then kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/quick
mkdir -p $OUT
echo "== tests" && timeout -k 10 400 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/bench.log 2>&1; rc=$?; cat $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/rocprof.log 2>&1 \
&& grep -E "aead|Name" $OUT/prof/run_kernel_stats.csv
