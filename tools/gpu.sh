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
#   ab               tools/ab.py over AB_LIBS (variant .so paths; AB_PAD / AB_BURST / AB_ROUNDS)
#   ab-full          config 2 and config 4 A/B of the build/variants names in AB_NAMES
#   power-ab         seal-only A/B of AB_NAMES, then each alone under tools/power_probe.py
#   pmc-sizes        HBM traffic of the descriptor kernels per payload size (config 3, one size at a time)
#   pmc-cmd          the generic PMC passes (one rocprofv3 run per counter group) over PMC_CMD
#   profile          bench lines for configs PROFILE_CONFIGS (2 3 4), kernel traces, the neptun
#                    layout line + trace, PMC traffic and VALU per config
#   cpu-scaling      the CPU baseline's thread scaling on this host (unpinned, packed, spread)
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
    ab) run 600 "$OUT/ab.log" env AB_PAD="${AB_PAD:-1}" AB_BURST="${AB_BURST:-100}" AB_ROUNDS="${AB_ROUNDS:-6}" \
          python tools/ab.py ${AB_LIBS:?AB_LIBS: variant .so paths} ;;
    ab-full)
      libs=""; for v in ${AB_NAMES:?AB_NAMES: build/variants names}; do libs="$libs build/variants/libneptun_gpu_$v.so"; done
      run 400 "$OUT/ab_config2.log" env AB_PAD=1 AB_BURST="${AB_BURST:-300}" AB_ROUNDS="${AB_ROUNDS:-10}" python tools/ab.py $libs
      run 400 "$OUT/ab_config4.log" env AB_CONFIG=4 AB_BURST=20 AB_ROUNDS=6 python tools/ab.py $libs ;;
    power-ab)
      libs=""; for v in ${AB_NAMES:?AB_NAMES: build/variants names}; do libs="$libs build/variants/libneptun_gpu_$v.so"; done
      run 400 "$OUT/ab_seal.log" env AB_SEAL_ONLY=1 AB_PAD=1 AB_BURST="${AB_BURST:-600}" AB_ROUNDS="${AB_ROUNDS:-6}" \
        python tools/ab.py $libs
      for v in $AB_NAMES; do
        run 120 "$OUT/power_$v.log" env AB_SEAL_ONLY=1 AB_BURST=1500 AB_ROUNDS=3 python tools/power_probe.py \
          "$OUT/power_$v.json" -- python tools/ab.py "build/variants/libneptun_gpu_$v.so"
      done ;;
    pmc-sizes)
      for spec in 64:1048576 256:1048576 576:524288 1350:262144 8900:65536; do
        P=${spec%%:*}; N=${spec##*:}
        run 300 "$OUT/pmc_size$P.log" python tools/pmc_traffic.py "$OUT/pmc_traffic_size$P.json" --config 3 \
          --mixed-sizes "$P" --per-size "$N"
      done ;;
    pmc-cmd)
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
                 "FETCH_SIZE" "WRITE_SIZE" \
                 "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS TCC_HIT TCC_MISS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM"; do
        i=$((i+1))
        run 300 "$OUT/pmc_p$i.log" rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_p$i" -o pmc -- \
          ${PMC_CMD:?PMC_CMD: the program, e.g. python3 bench.py --no-cpu-baseline}
      done ;;
    profile)
      python3 -c "import bench, json; print(json.dumps(bench.host_cpus()))" > "$OUT/host_cpus.json"
      for c in ${PROFILE_CONFIGS:-2 3 4}; do
        run 300 "$OUT/bench_config$c.json" python3 bench.py --config "$c" --steps 20 --warmup 5
      done
      run 300 "$OUT/trace_bench_config2.json" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" \
        -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-seconds 0
      run 300 "$OUT/bench_config2_neptun.json" python3 bench.py --layout neptun --steps 20 --warmup 5 --no-cpu-baseline
      run 300 "$OUT/trace_bench_config2_neptun.json" rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/trace_neptun" -o run -- python3 bench.py --layout neptun --steps 20 --warmup 5 --no-cpu-baseline \
        --sustain-seconds 0
      run 400 "$OUT/pmc_neptun.log" python3 tools/pmc_traffic.py "$OUT/pmc_traffic_config2_neptun.json" --layout neptun
      for c in ${PROFILE_CONFIGS:-2 3 4}; do
        run 400 "$OUT/pmc_traffic_config$c.log" python3 tools/pmc_traffic.py "$OUT/pmc_traffic_config$c.json" --config "$c"
        run 400 "$OUT/pmc_valu_config$c.log" python3 tools/pmc_valu.py "$OUT/pmc_valu_config$c.json" --config "$c"
      done ;;
    cpu-scaling)
      E=oracle/build/cpu_baseline
      {
        echo "nproc=$(nproc) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
        grep -m1 "model name" /proc/cpuinfo
        for t in 1 2 4 8 16; do
          echo "unpinned t=$t: $(timeout 120 $E --impl openssl --threads $t --packets $((65536 * t)) --reps 7)"
        done
        for t in 1 4 8 12 16; do
          echo "packed t=$t: $(timeout 120 taskset -c $(seq -s, 0 $((t - 1))) $E --impl openssl --threads $t \
            --packets $((65536 * t)) --reps 7)"
        done
      } > "$OUT/cpu_scaling.txt" 2>&1
      cat "$OUT/cpu_scaling.txt" ;;
    cmd=*) run 600 "$OUT/cmd_$(date +%s).txt" bash -c "${step#cmd=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== $TAG: all steps passed"
