#!/bin/bash
# Small Tunn calls under host-side knobs (pool grains, event-wait spin), interleaved A/B:
#   tools/ab_grain.sh TAG "NAME:ENV=V,ENV=V" ...   (outputs gpurun_out/TAG/NAME_{reg,staged}_R.jsonl)
set -e
TAG=${1:?}; shift
mkdir -p gpurun_out/$TAG
B="python tools/bench_tunn.py --sizes ${AB_SIZES:-16,64,128,256,512,1024,4096} --reps 30 ${AB_FLAGS---phase-timing}"
for r in $(seq 1 ${AB_REPS:-2}); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    for mode in reg staged; do
      flag=; [ $mode = reg ] && flag=--register
      env ${envs//,/ } timeout -k 10 150 $B $flag > gpurun_out/$TAG/${name}_${mode}_$r.jsonl
    done
  done
done
