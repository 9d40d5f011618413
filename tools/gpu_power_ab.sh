#!/bin/bash
# Seal-only A/B of variant builds plus a power / clock probe per variant (run via
# gpurun).  Seal-only bursts keep timing ablations honest: an ablated variant's
# open fails its tag check and zero-fills, which draws a different power than a
# real open and would shift the clock of the next seal.
#   tools/gpu_power_ab.sh TAG name...   (build/variants/libneptun_gpu_<name>.so; outputs gpurun_out/TAG/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
V=build/variants
libs=()
for v in "$@"; do libs+=("$V/libneptun_gpu_$v.so"); done
AB_SEAL_ONLY=1 AB_BURST=${AB_BURST:-600} AB_ROUNDS=${AB_ROUNDS:-6} bash tools/gpu_probe.sh "$TAG" "${libs[@]}" || exit $?
for v in "$@"; do
  AB_SEAL_ONLY=1 AB_BURST=1500 AB_ROUNDS=3 timeout -k 10 120 python tools/power_probe.py "$OUT/power_$v.json" -- \
    python tools/ab.py "$V/libneptun_gpu_$v.so" > "$OUT/power_$v.log" 2>&1 || exit $?
  python -c "import json;d=json.load(open('$OUT/power_$v.json'));print('$v',d['summary'])"
done
