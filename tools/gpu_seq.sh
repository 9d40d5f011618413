#!/bin/bash
# tests then A/B:  tools/gpu_seq.sh variant.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/seq
echo "== tests" && timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/seq/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/seq/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== ab" && timeout -k 10 600 python tools/ab.py "$@" > gpurun_out/seq/ab.log 2>&1; rc=$?; cat gpurun_out/seq/ab.log; exit $rc
