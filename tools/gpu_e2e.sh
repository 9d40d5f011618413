#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/e2e; mkdir -p $OUT

timeout -k 10 600 python tools/bench_e2e.py > $OUT/e2e.jsonl 2> $OUT/e2e.err; rc=$?; cat $OUT/e2e.jsonl; exit $rc
