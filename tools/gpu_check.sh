#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== tests" && timeout -k 10 400 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log \
&& echo "== bench" && timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && cat $OUT/bench.log \
&& echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/rocprof.log 2>&1 \
&& find $OUT/prof -name "*stats*" | head && cat $(find $OUT/prof -name "*kernel_stats.csv" | head -1)
