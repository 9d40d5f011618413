set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 build/proto/microbench_dma 1350 > gpurun_out/r04g_dma.jsonl
for v in product k4; do
  timeout -k 10 60 python tools/power_probe.py gpurun_out/r04g_power_$v.json -- python tools/proto_xlane.py loop $v --seconds 5 > gpurun_out/r04g_power_$v.log
done
