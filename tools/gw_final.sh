#!/bin/bash
# gateway sweep on the final tree: batches 50 .. 16384, 1-8 pairs, GPU (plain and
# registered pools) beside the CPU line, 3 runs (medians: tools/gw_table.py --median)
set -e
mkdir -p gpurun_out/$1
for r in 1 2 3; do
  GW_BACKEND="gpu cpu" GW_PAIRS="1 2 4 8" GW_REG="0 1" timeout -k 10 500 python tools/bench_gateway.py 262144 1350 50 256 1024 4096 16384 > gpurun_out/$1/final_$r.jsonl
done
