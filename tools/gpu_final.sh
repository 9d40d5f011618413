#!/bin/bash
# Round-end rehearsal (run via gpurun): the GPU test suite, smoke(), the bench as
# the driver runs it (N=1, and through torch.distributed.run with one rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
echo "== tests" && timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log \
&& echo "== bench" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && cut -c1-400 $OUT/bench.json \
&& echo "== torchrun n=1" && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_torchrun.json 2> $OUT/bench_torchrun.err && cut -c1-400 $OUT/bench_torchrun.json
