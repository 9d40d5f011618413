#!/bin/bash
# One GPU-box session made of named steps:
#   tools/gpu.sh TAG STEP [STEP ...]
# Outputs go to gpurun_out/TAG/.  Every step runs under its own time limit and the
# first failing step ends the call (no retries).  Steps:
#   tests            the whole GPU suite (pytest -m gpu)
#   test=FILE[,..]   the named test files only (tests/FILE)
#   smoke            __graft_entry__.smoke()
#   bench[=CFG]      bench.py (default config 2) -> bench_CFG.json
#   trace            rocprofv3 kernel trace + stats of bench.py -> trace/
#   pmc              tools/pmc_traffic.py (HBM bytes per launch, separate --pmc passes)
#   valu             tools/pmc_valu.py
#   xlane            tools/bench_xlane.py: latency vs throughput forms, 1 .. 16384 packets
#   tunn-small       tools/bench_tunn.py at 64 .. 16384 packets (staged and registered)
#   tunn-big         tools/bench_tunn.py at 262144 packets (registered)
#   gateway          tools/bench_gateway.py sweep (GW_ARGS overrides its arguments)
#   cmd=...          any other command line (quoted by the caller; runs under a 600 s limit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?usage: tools/gpu.sh TAG STEP [STEP ...]}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"

run() {  # run LIMIT LOG CMD...: one step, its output in LOG, ends the call on failure
  local limit=$1 log=$2
  shift 2
  echo "== $TAG: $* (limit ${limit}s) -> $log"
  timeout -k 10 "$limit" "$@" > "$log" 2>&1
  local rc=$?
  tail -6 "$log"
  if [ $rc -ne 0 ]; then
    echo "== $TAG: step failed rc=$rc"
    exit $rc
  fi
}

for step in "$@"; do
  case "$step" in
    tests) run 900 "$OUT/pytest_gpu.txt" $PYT tests -m gpu ;;
    test=*)
      files=""
      for f in $(echo "${step#test=}" | tr ',' ' '); do files="$files tests/$f"; done
      run 600 "$OUT/pytest_$(echo "${step#test=}" | tr ',/' '__').txt" $PYT $files ;;
    smoke) run 180 "$OUT/smoke.txt" python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 400 "$OUT/bench_2.json" python bench.py ;;
    bench=*) run 600 "$OUT/bench_${step#bench=}.json" python bench.py --config "${step#bench=}" ;;
    trace)
      run 400 "$OUT/trace_bench.json" rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
        --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    pmc) run 900 "$OUT/pmc.log" python tools/pmc_traffic.py "$OUT/pmc_traffic.json" ;;
    valu) run 600 "$OUT/valu.log" python tools/pmc_valu.py "$OUT/pmc_valu.json" ;;
    xlane) run 300 "$OUT/xlane.jsonl" python tools/bench_xlane.py ${XLANE_ARGS:-} ;;
    tunn-small)
      run 300 "$OUT/tunn_small.jsonl" python tools/bench_tunn.py --sizes 64,256,1024,4096,16384 --reps 30 --phase-timing
      run 300 "$OUT/tunn_small_reg.jsonl" python tools/bench_tunn.py --sizes 64,256,1024,4096,16384 --reps 30 \
        --phase-timing --register ;;
    tunn-big) run 300 "$OUT/tunn_big.jsonl" python tools/bench_tunn.py --sizes 262144 --reps 7 --phase-timing --register ;;
    gateway) run 900 "$OUT/gateway.jsonl" python tools/bench_gateway.py ${GW_ARGS:-} ;;
    cmd=*) run 600 "$OUT/cmd_$(date +%s).txt" bash -c "${step#cmd=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== $TAG: all steps passed"
