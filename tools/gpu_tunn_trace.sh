#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tunn
WG_TUNN_TRACE=1 WG_TUNN_CHUNK_KB=16384 timeout -k 10 120 python tools/bench_tunn.py --sizes 65536 --reps 3 > gpurun_out/tunn/trace.out 2> gpurun_out/tunn/trace.err; rc=$?; cat gpurun_out/tunn/trace.out; tail -40 gpurun_out/tunn/trace.err; exit $rc
