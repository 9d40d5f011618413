#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/diag4
timeout -k 10 200 ./tools/microbench_valu > gpurun_out/diag4/valu.txt 2>&1 || exit 1
AB_ROUNDS=1 ./tools/pmc.sh gpurun_out/diag4/pmc_e -- python3 tools/ab.py build/variants/libneptun_gpu_e.so
