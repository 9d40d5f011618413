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
#   tunn-ab          small Tunn calls, staged and registered, AB_REPS (3) interleaved runs of
#                    every variant in AB_VARIANTS ("NAME:ENV=V,ENV=V ...", default "base:X=1")
#                    at AB_SIZES (1..4096) with bench_tunn.py flags AB_FLAGS (none)
#                    -> NAME_{reg,staged}_R.jsonl (table: tools/ab_grain_table.py)
#   tt-ab            concurrent small calls without sockets: build/probes/tunn_threads at
#                    T = 1 and 8 threads, batch TT_BATCH (50), per AB_VARIANTS -> tt_NAME.jsonl
#   gw-ab            gateway GPU + CPU lines at GW_BATCHES ("50 256"), 1-8 pairs, plain and
#                    registered pools, 3 runs, then AB_VARIANTS on the GPU line
#                    -> base_R.jsonl, NAME_R.jsonl (table: tools/gw_table.py DIR base --median)
#   launch-latency   build/probes/launch_latency (completion mechanisms, multi-thread rates)
#   cmd=...          any other command line (quoted by the caller; runs under a 600 s limit)
# (build/probes/*: gcc -O2 -pthread -DTT_ENGINES -Iinclude tools/tunn_threads.c -Lneptun_amd
#  -lneptun_gpu -Wl,-rpath,'$ORIGIN/../../neptun_amd' -o build/probes/tunn_threads;
#  hipcc --offload-arch=gfx950 -O2 tools/probes/launch_latency.cpp -o build/probes/launch_latency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?usage: tools/gpu.sh TAG STEP [STEP ...]}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"

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
    tunn-ab)
      for r in $(seq 1 "${AB_REPS:-3}"); do
        for v in ${AB_VARIANTS:-base:X=1}; do
          name=${v%%:*}; envs=${v#*:}
          for mode in reg staged; do
            flag=; [ $mode = reg ] && flag=--register
            run 200 "$OUT/${name}_${mode}_$r.jsonl" env ${envs//,/ } python tools/bench_tunn.py \
              --sizes "${AB_SIZES:-1,16,50,64,128,256,1024,4096}" --reps 30 ${AB_FLAGS:-} $flag
          done
        done
      done ;;
    tt-ab)
      for v in ${AB_VARIANTS:-base:X=1}; do
        name=${v%%:*}; envs=${v#*:}
        for T in 1 8; do
          run 60 "$OUT/tt_${name}_T$T.jsonl" env ${envs//,/ } build/probes/tunn_threads $T "${TT_BATCH:-50}" 2000 1350
        done
        cat "$OUT"/tt_${name}_T*.jsonl > "$OUT/tt_$name.jsonl"
      done ;;
    gw-ab)
      for r in 1 2 3; do
        run 500 "$OUT/base_$r.jsonl" env GW_BACKEND="gpu cpu" GW_PAIRS="1 2 4 8" GW_REG="0 1" \
          python tools/bench_gateway.py 262144 1350 ${GW_BATCHES:-50 256}
        for v in ${AB_VARIANTS:-}; do
          name=${v%%:*}; envs=${v#*:}
          run 500 "$OUT/${name}_$r.jsonl" env ${envs//,/ } GW_PAIRS="1 2 4 8" GW_REG="0 1" \
            python tools/bench_gateway.py 262144 1350 ${GW_BATCHES:-50 256}
        done
      done ;;
    launch-latency) run 120 "$OUT/launch_latency.json" build/probes/launch_latency ;;
    cmd=*) run 600 "$OUT/cmd_$(date +%s).txt" bash -c "${step#cmd=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== $TAG: all steps passed"
