#!/bin/bash
# tt_ab_lib.sh OUTDIR name=libdir[:ENV=V,ENV=V] ... -- small-call A/B of builds of
# libneptun_gpu.so (and of environment knobs):
# build/probes/tunn_threads (8 and 1 threads, 50 x 1350 B, staged and registered) run
# against each library directory in turn (LD_LIBRARY_PATH over the probe's runpath),
# ROUNDS (3) rounds alternating, one JSON line per run in OUTDIR/tt_<name>_T<T>_R<reg>.jsonl.
set -e
out=$1; shift
mkdir -p "$out"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for v in "$@"; do
    name=${v%%=*}; lib=${v#*=}; envs=
    case $lib in *:*) envs=${lib#*:}; lib=${lib%%:*} ;; esac
    for T in 1 8; do
      for reg in 0 1; do
        env ${envs//,/ } LD_LIBRARY_PATH=$lib TT_REGISTER=$reg timeout -k 10 60 build/probes/tunn_threads $T 50 "${CALLS:-10000}" 1350 \
          >> "$out/tt_${name}_T${T}_R${reg}.jsonl"
      done
    done
  done
  echo "round $r done"
done
