#!/bin/bash
# Round 4: the reference's own AEAD bench shape (chacha20poly1305_benching.rs:37-55):
# config-2 lines at 128 / 192 / 1400 / 8192 B, seal-only and open-only, each with the CPU
# baseline at the same size, plus one rocprofv3 kernel trace per size.
# usage: tools/gpu_r04_sizes.sh TAG   (outputs under gpurun_out/TAG_*)
set -euo pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for P in 128 192 1400 8192; do
  for OP in seal open; do
    timeout -k 10 240 python bench.py --size $P --op $OP --steps 20 --warmup 5 --cpu-curve "" \
      > gpurun_out/${TAG}_bench_p${P}_${OP}.json 2> gpurun_out/${TAG}_bench_p${P}_${OP}.err
  done
  timeout -k 10 240 python bench.py --size $P --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/${TAG}_bench_p${P}_roundtrip.json 2> gpurun_out/${TAG}_bench_p${P}_roundtrip.err
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_p${P} -o run -- \
    python bench.py --size $P --steps 20 --warmup 5 --no-cpu-baseline --sustain-seconds 0 \
    > gpurun_out/${TAG}_prof_p${P}.log 2>&1
done
