#!/bin/bash
# Round-3 probe (run via gpurun): text-grid open vs wire-grid open (NepTUN's
# decapsulate layout), descriptor-kernel variants on config 4, the new bench
# fields, and PMC traffic of the NepTUN-layout line.  Outputs gpurun_out/$TAG/.
#   tools/gpu_r03_probe.sh TAG [variant...]   (build/variants/libneptun_gpu_<v>.so; first = reference)
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
step() {  # step NAME SECONDS cmd...  (stdout+stderr to $OUT/NAME.log)
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -n 12 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "== $name failed rc=$rc"; exit $rc; }
}
if [ -n "$PROBE_TEXT" ]; then
  step text_grid 300 env AB_PAD=0 AB_OPEN_OFF=0 AB_BURST=100 AB_ROUNDS=6 python tools/ab.py "${libs[@]}"
  step wire_grid 200 env AB_PAD=0 AB_OPEN_OFF=16 AB_BURST=100 AB_ROUNDS=4 python tools/ab.py "${libs[0]}"
fi
if [ -n "$PROBE_C4" ]; then
  step config4 400 env AB_CONFIG=4 AB_PER_PEER=1024 AB_BURST=6 AB_ROUNDS=6 python tools/ab.py "${libs[@]}"
  step config4_one_peer 300 env AB_CONFIG=4 AB_PEERS=1 AB_PER_PEER=4194304 AB_BURST=6 AB_ROUNDS=6 python tools/ab.py "${libs[0]}"
fi
if [ -n "$PROBE_BENCH" ]; then
  step bench_config2 300 python bench.py --steps 20 --warmup 5
  step bench_neptun 300 python bench.py --layout neptun --steps 20 --warmup 5 --no-cpu-baseline
fi
if [ -n "$PROBE_PMC_NEPTUN" ]; then
  step pmc_traffic_neptun 400 python tools/pmc_traffic.py "$OUT/pmc_traffic_config2_neptun.json" --layout neptun
fi
if [ -n "$PROBE_POWER" ]; then  # seal-only A/B + power probe per variant ($PROBE_POWER = variants)
  step power_ab 900 bash tools/gpu_power_ab.sh "$TAG/power" $PROBE_POWER
fi
if [ -n "$PROBE_C4_BENCH" ]; then
  step bench_config4 600 python bench.py --config 4 --steps 10 --warmup 3 --sustain-seconds 6
fi
if [ -n "$PROBE_C4_SHAPE" ]; then  # what makes config 4 slower: footprint, per-lane keys or the kernel
  step c2_1m 200 env AB_PAD=0 AB_OPEN_OFF=16 AB_BURST=100 AB_ROUNDS=4 python tools/ab.py "${libs[0]}"
  step c4_1m_1peer 300 env AB_CONFIG=4 AB_PEERS=1 AB_PER_PEER=1048576 AB_BURST=40 AB_ROUNDS=5 python tools/ab.py "${libs[0]}"
  step c4_1m_4096peers 300 env AB_CONFIG=4 AB_PEERS=4096 AB_PER_PEER=256 AB_BURST=40 AB_ROUNDS=5 python tools/ab.py "${libs[0]}"
  step c4_16m_1peer 600 env AB_CONFIG=4 AB_PEERS=1 AB_PER_PEER=16777216 AB_BURST=3 AB_ROUNDS=4 python tools/ab.py "${libs[0]}"
  step c2_16m 400 python bench.py --packets 16777216 --steps 5 --warmup 2 --sustain-seconds 3 --no-cpu-baseline --evp-sample 0
fi
echo "== done"
