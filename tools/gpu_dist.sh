#!/bin/bash
# Rehearsal of the multi-rank bench path on a one-GPU box: 2 ranks share the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/dist; mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/bench2r.json 2> $OUT/bench2r.err; rc=$?; cat $OUT/bench2r.json; tail -3 $OUT/bench2r.err; exit $rc
