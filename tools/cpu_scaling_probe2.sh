#!/bin/bash
# CPU-baseline scaling on the GPU box's host, round 2 (no GPU use): 64 Ki packets PER
# THREAD, threads pinned one per physical core -- packed (cpus 0..t-1, adjacent
# cores) and spread (every 8th core: one per CCD first) -- at 1..16 threads, to see
# where the job's 16-CPU quota (cgroup cpu.max 1600000/100000) starts throttling.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
E=oracle/build/cpu_baseline
{
  for t in 1 2 4 8 12 14 15 16; do
    cpus=$(seq -s, 0 $((t - 1)))
    echo "packed t=$t: $(timeout 120 taskset -c $cpus $E --impl openssl --threads $t --packets $((65536 * t)) --reps 7)"
  done
  for t in 4 8 12 14 16; do
    cpus=$(for i in $(seq 0 $((t - 1))); do echo -n "$(( (i * 8) % 128 + (i * 8) / 128 )),"; done)
    cpus=${cpus%,}
    echo "spread cpus=$cpus t=$t: $(timeout 120 taskset -c $cpus $E --impl openssl --threads $t --packets $((65536 * t)) --reps 7)"
  done
  grep -E "nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null
} > $OUT/cpu_scaling2.txt 2>&1
cat $OUT/cpu_scaling2.txt
