#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB_ROUNDS=1 ./tools/pmc.sh gpurun_out/diag3/pmc_b -- python3 tools/ab.py build/variants/libneptun_gpu_b.so
