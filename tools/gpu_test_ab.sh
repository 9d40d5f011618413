#!/bin/bash
# GPU parity tests (optionally filtered by $TESTK) then an A/B of variant builds:
#   tools/gpu_test_ab.sh build/variants/a.so build/variants/b.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/tab
mkdir -p $OUT
K=${TESTK:+-k "$TESTK"}
echo "== tests" && eval timeout -k 10 900 python -m pytest tests -x -q -m gpu $K > $OUT/pytest.log 2>&1; rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
[ $# -eq 0 ] && exit 0
echo "== ab" && timeout -k 10 600 python tools/ab.py "$@" > $OUT/ab.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/ab.log; exit $rc
