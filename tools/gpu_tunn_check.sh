#!/bin/bash
# Tunn batch parity tests, then the Tunn host-path benchmark (staged and registered).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tunn
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "tunn or replay" > gpurun_out/tunn/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/tunn/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_tunn.py "$@" > gpurun_out/tunn/bench.jsonl 2> gpurun_out/tunn/bench.err; rc=$?; cat gpurun_out/tunn/bench.jsonl; tail -3 gpurun_out/tunn/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_tunn.py --register "$@" > gpurun_out/tunn/bench_reg.jsonl 2> gpurun_out/tunn/bench_reg.err; rc=$?; cat gpurun_out/tunn/bench_reg.jsonl; tail -3 gpurun_out/tunn/bench_reg.err; exit $rc
