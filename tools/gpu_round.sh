#!/bin/bash
# Full GPU session: parity tests, smoke, bench (configs 2/3/4), kernel trace, PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
step() { echo "== $1"; }
step tests && timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step smoke && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log \
&& step bench2 && timeout -k 10 400 python bench.py > $OUT/bench2.json 2> $OUT/bench2.err && cat $OUT/bench2.json \
&& step bench3 && timeout -k 10 400 python bench.py --config 3 --steps 20 > $OUT/bench3.json 2> $OUT/bench3.err && cat $OUT/bench3.json \
&& step bench4 && timeout -k 10 600 python bench.py --config 4 --steps 5 --warmup 2 > $OUT/bench4.json 2> $OUT/bench4.err && cat $OUT/bench4.json \
&& step trace && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.log && cat $OUT/trace_bench.json \
&& grep -E "aead|Name" $OUT/trace/run_kernel_stats.csv \
&& step pmc && timeout -k 10 900 python tools/pmc_traffic.py $OUT/pmc_traffic.json > $OUT/pmc.log 2>&1 && cat $OUT/pmc_traffic.json \
&& step valu && timeout -k 10 600 python tools/pmc_valu.py $OUT/pmc_valu.json > $OUT/valu.log 2>&1 && cat $OUT/pmc_valu.json
