#!/bin/bash
# gateway at NepTUN's batch sizes (50, 256): GPU line (this build, and with the knobs in
# "$@" as NAME:ENV=V,...) beside the CPU line, 1-8 pairs, plain and registered pools, 3 runs
set -e
TAG=${1:?}; shift
mkdir -p gpurun_out/$TAG
for r in 1 2 3; do
  GW_BACKEND="gpu cpu" GW_PAIRS="1 2 4 8" GW_REG="0 1" timeout -k 10 300 python tools/bench_gateway.py 262144 1350 50 256 > gpurun_out/$TAG/base_$r.jsonl
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } GW_PAIRS="1 2 4 8" GW_REG="0 1" timeout -k 10 300 python tools/bench_gateway.py 262144 1350 50 256 > gpurun_out/$TAG/${name}_$r.jsonl
  done
done
