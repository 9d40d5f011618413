#!/bin/bash
# Round-3 check (run via gpurun): the GPU suite on the product build, the
# non-phase-locked build (WG_SYNC=0) through the strided / slot-padding tests, and
# the text-grid alignment probe.  Outputs gpurun_out/$TAG/.
#   tools/gpu_r03_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {  # step NAME SECONDS cmd...  (stdout+stderr to $OUT/NAME.log)
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$OUT/$name.log" | tail -n 14
  [ $rc -eq 0 ] || { echo "== $name failed rc=$rc"; exit $rc; }
}
if [ -z "$SKIP_SUITE" ]; then
  step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
fi
if [ -n "$CHECK_NOSYNC" ]; then
  # this box's scratch copy only: the WG_SYNC=0 build in place of the product for the strided tests
  cp neptun_amd/libneptun_gpu.so "$OUT/product.so.bak" &&
    cp build/variants/libneptun_gpu_nosync.so neptun_amd/libneptun_gpu.so || exit 1
  step pytest_nosync 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "strided or padding" --timeout 120 --timeout-method thread
  cp "$OUT/product.so.bak" neptun_amd/libneptun_gpu.so && rm -f "$OUT/product.so.bak" || exit 1
fi
if [ -n "$CHECK_TEXT_ALIGN" ]; then
  V=build/variants
  step text_misaligned 200 env AB_PAD=0 AB_STRIDE=1536 AB_WIRE_OFF=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_base.so
  step text_aligned 200 env AB_PAD=0 AB_STRIDE=1536 AB_WIRE_OFF=112 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_base.so
  step wire_grid 200 env AB_PAD=0 AB_STRIDE=1536 AB_WIRE_OFF=0 AB_OPEN_OFF=16 AB_BURST=100 AB_ROUNDS=5 python tools/ab.py $V/libneptun_gpu_base.so
fi
if [ -n "$CHECK_DESC" ]; then  # descriptor-kernel variants ($CHECK_DESC), configs 4 and 3
  libs=()
  for v in $CHECK_DESC; do libs+=("build/variants/libneptun_gpu_$v.so"); done
  step desc_config4 400 env AB_CONFIG=4 AB_PER_PEER=1024 AB_BURST=6 AB_ROUNDS=6 python tools/ab.py "${libs[@]}"
  step desc_config3 400 env AB_CONFIG=3 AB_BURST=6 AB_ROUNDS=6 python tools/ab.py "${libs[@]}"
fi
if [ -n "$CHECK_PMC" ]; then  # HBM traffic of the descriptor configs with the current build
  for c in $CHECK_PMC; do
    step pmc_traffic_config$c 500 python tools/pmc_traffic.py "$OUT/pmc_traffic_config$c.json" --config $c
  done
fi
echo "== done"
