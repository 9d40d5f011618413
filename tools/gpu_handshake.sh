#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/hs; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k handshake > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_handshake.py > $OUT/bench.jsonl 2> $OUT/bench.err; rc=$?; cat $OUT/bench.jsonl; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/bench_handshake.py > $OUT/trace_bench.jsonl 2> $OUT/trace.err; rc=$?; grep -E "x25519|handshake|Name" $OUT/trace/run_kernel_stats.csv; exit $rc
