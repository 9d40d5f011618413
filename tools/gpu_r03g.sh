# round-3 session g: the final descriptor build -- suite, masked vs generic edge rounds,
# evidence refresh for configs 3 / 4 (+ the config-2 trace), per-size traffic of config 3
CHECK_DESC="base masked" bash tools/gpu_r03_check.sh r03g \
  && bash tools/gpu_profile.sh r03g_prof 3 4 \
  && bash tools/gpu_pmc_sizes.sh r03g_sizes
