#!/bin/bash
# CPU-baseline scaling on the GPU box's host (no GPU use): the job's CPU share as the
# kernel sees it, then oracle/build/cpu_baseline at 1..16 threads -- unpinned, and
# pinned to distinct physical cores -- outside any python/HIP process.
# Outputs gpurun_out/$TAG/cpu_scaling.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
{
  echo "nproc=$(nproc) OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"
  echo "cgroup=$(cat /proc/self/cgroup 2>/dev/null | head -3 | tr '\n' ' ')"
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/cpu.weight; do
    [ -r $f ] && echo "$f: $(cat $f)"
  done
  grep -m1 "model name" /proc/cpuinfo
  echo "siblings of cpu0: $(cat /sys/devices/system/cpu/cpu0/topology/thread_siblings_list 2>/dev/null)"
  E=oracle/build/cpu_baseline
  for t in 1 2 4 8 16; do
    echo "unpinned t=$t packets=65536: $(timeout 120 $E --impl openssl --threads $t --packets 65536 --reps 11)"
  done
  for t in 1 4 16; do
    echo "unpinned t=$t packets=$((65536 * t)): $(timeout 120 $E --impl openssl --threads $t --packets $((65536 * t)) --reps 7)"
  done
  # one CPU per physical core: the first SMT sibling of cores 0..15 (cpu i on this layout)
  for t in 1 4 16; do
    cpus=$(seq -s, 0 $((t - 1)))
    echo "pinned cpus=$cpus t=$t packets=$((65536 * t)): $(timeout 120 taskset -c $cpus $E --impl openssl --threads $t --packets $((65536 * t)) --reps 7)"
  done
} > $OUT/cpu_scaling.txt 2>&1
cat $OUT/cpu_scaling.txt
