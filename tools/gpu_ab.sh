#!/bin/bash
# A/B timing of variant builds in one process:  tools/gpu_ab.sh build/variants/*.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python tools/ab.py "$@" > gpurun_out/ab/ab.log 2>&1; rc=$?; cat gpurun_out/ab/ab.log; exit $rc
