#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/cfg3; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k "plan or mixed or config3" > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 3 --steps 20 > $OUT/bench3.json 2> $OUT/bench3.err && cat $OUT/bench3.json
