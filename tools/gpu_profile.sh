#!/bin/bash
# One GPU-box pass that refreshes the measurement evidence (run via gpurun):
#   bench lines for configs 2-4, the rocprofv3 kernel-trace summary of the
#   config-2 bench command, and the PMC traffic / VALU summaries per config
#   (separate rocprofv3 passes, never combined with tracing domains).
# Usage: tools/gpu_profile.sh TAG [configs...]    (outputs under gpurun_out/TAG/)
set -euo pipefail
TAG=${1:?tag}
shift
CONFIGS=${*:-2 3 4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import bench, json; print(json.dumps(bench.host_cpus()))" > "$OUT/host_cpus.json"
for c in $CONFIGS; do
  timeout -k 10 300 python3 bench.py --config "$c" --steps 20 --warmup 5 > "$OUT/bench_config$c.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sustain-seconds 0 > "$OUT/trace_bench_config2.json"
# NepTUN's own buffer layouts (seal in place, open to offset 0: the text grid)
timeout -k 10 300 python3 bench.py --layout neptun --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_config2_neptun.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_neptun" -o run -- \
  python3 bench.py --layout neptun --steps 20 --warmup 5 --no-cpu-baseline --sustain-seconds 0 > "$OUT/trace_bench_config2_neptun.json"
timeout -k 10 400 python3 tools/pmc_traffic.py "$OUT/pmc_traffic_config2_neptun.json" --layout neptun > /dev/null
for c in $CONFIGS; do
  timeout -k 10 400 python3 tools/pmc_traffic.py "$OUT/pmc_traffic_config$c.json" --config "$c" > /dev/null
  timeout -k 10 400 python3 tools/pmc_valu.py "$OUT/pmc_valu_config$c.json" --config "$c" > /dev/null
done
echo "done $TAG"
