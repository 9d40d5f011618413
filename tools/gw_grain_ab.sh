#!/bin/bash
# gateway sweep (batches 50 .. 4096, 1-8 pairs, plain and registered pools) with the pool
# grains of this build vs the previous ones, interleaved
set -e
mkdir -p gpurun_out/$1
for r in 1 2; do
  GW_PAIRS="1 2 4 8" GW_REG="0 1" timeout -k 10 300 python tools/bench_gateway.py 262144 1350 50 256 1024 4096 > gpurun_out/$1/new_$r.jsonl
  WG_TUNN_GRAIN_LIGHT=64 WG_TUNN_COPY_SPLIT=1 GW_PAIRS="1 2 4 8" GW_REG="0 1" timeout -k 10 300 python tools/bench_gateway.py 262144 1350 50 256 1024 4096 > gpurun_out/$1/old_$r.jsonl
done
