#!/bin/bash
# A/B of two or more variant builds on configs 2 and 4 (round trips, correct
# outputs), then the GPU parity suites on the in-tree product build.
#   tools/gpu_ab_full.sh TAG name...   (build/variants/libneptun_gpu_<name>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
libs=()
for v in "$@"; do libs+=("build/variants/libneptun_gpu_$v.so"); done
AB_PAD=1 AB_BURST=${AB_BURST:-300} AB_ROUNDS=${AB_ROUNDS:-10} timeout -k 10 400 python tools/ab.py "${libs[@]}" > "$OUT/ab_config2.log" 2>&1 || { cat "$OUT/ab_config2.log"; exit 1; }
grep -E "med|round-trip" "$OUT/ab_config2.log"
AB_CONFIG=4 AB_BURST=20 AB_ROUNDS=6 timeout -k 10 400 python tools/ab.py "${libs[@]}" > "$OUT/ab_config4.log" 2>&1 || { cat "$OUT/ab_config4.log"; exit 1; }
grep -E "med|round-trip" "$OUT/ab_config4.log"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -2 "$OUT/pytest_gpu.log"
exit $rc
