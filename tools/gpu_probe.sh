#!/bin/bash
# Same-box bound probes: tools/ab.py over variant builds, then the staging
# microbenchmark.  Usage: tools/gpu_probe.sh TAG variant.so...   (gpurun_out/TAG/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
AB_PAD=${AB_PAD:-1} AB_BURST=${AB_BURST:-100} AB_ROUNDS=${AB_ROUNDS:-6} \
  timeout -k 10 400 python tools/ab.py "$@" > "$OUT/ab.log" 2>&1; rc=$?
cat "$OUT/ab.log"
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROBE_MEM4" ]; then
  timeout -k 10 200 ./tools/probes/microbench_mem4 > "$OUT/mem4.log" 2>&1; rc=$?
  cat "$OUT/mem4.log"
  exit $rc
fi
