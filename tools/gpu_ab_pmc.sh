#!/bin/bash
# A/B of variant builds (configs 2 and 4, then the GPU suite: tools/gpu_ab_full.sh)
# plus the PMC VALU-instruction count of the in-tree build's config-2 kernels.
#   tools/gpu_ab_pmc.sh TAG name...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:?tag}
bash tools/gpu_ab_full.sh "$@" || exit $?
timeout -k 10 400 python tools/pmc_valu.py "gpurun_out/$TAG/pmc_valu_config2.json" --config 2 > "gpurun_out/$TAG/pmc.log" 2>&1 || exit $?
cat "gpurun_out/$TAG/pmc_valu_config2.json"
