#!/bin/bash
# Round 3 (s): batched Tunn host path -- pipeline depth (WG_TUNN_SETS 2/3/4 staging
# sets) x chunk size, copy and registered buffers; Tunn GPU tests at depth 3 and 4.
# gpurun_out/r03s/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03s
mkdir -p $OUT
: > $OUT/tunn_sweep.jsonl
for sets in 2 3 4; do
  for kb in 8192 16384; do
    for reg in "" "--register"; do
      echo "{\"sets\": $sets, \"chunk_kb\": $kb, \"register\": \"$reg\"}" >> $OUT/tunn_sweep.jsonl
      WG_TUNN_SETS=$sets WG_TUNN_CHUNK_KB=$kb timeout -k 10 120 python3 tools/bench_tunn.py --sizes 65536,262144 --reps 7 $reg >> $OUT/tunn_sweep.jsonl 2>> $OUT/tunn_sweep.err || { echo "bench failed sets=$sets kb=$kb $reg"; tail -5 $OUT/tunn_sweep.err; exit 1; }
    done
  done
done
cat $OUT/tunn_sweep.jsonl
for sets in 3 4; do
  WG_TUNN_SETS=$sets timeout -k 10 300 python -u -m pytest tests/test_tunn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_tunn_sets$sets.log 2>&1 || { tail -20 $OUT/pytest_tunn_sets$sets.log; exit 1; }
  tail -1 $OUT/pytest_tunn_sets$sets.log
done
