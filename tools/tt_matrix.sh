#!/bin/bash
# concurrent small Tunn calls (tools/tunn_threads.c, no sockets) under host-path variants:
#   tools/tt_matrix.sh TAG B "NAME:ENV=V,..." ...  -> gpurun_out/TAG/NAME.jsonl (T = 1, 8)
set -e
TAG=${1:?}; B=${2:?}; shift 2
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  for T in 1 8; do env ${envs//,/ } timeout -k 10 60 build/probes/tunn_threads $T $B 2000 1350 >> gpurun_out/$TAG/$name.jsonl; done
done
