# round-3 session: suite + descriptor variants + rotate-form power A/B, then the evidence
# refresh of the current build (bench lines, kernel trace, PMC per config, handshake rates);
# each step under its own timeout, stop at the first failure
CHECK_DESC="base nofull ukey ukeynf" bash tools/gpu_r03_check.sh r03f \
  && bash tools/gpu_power_ab.sh r03f/power base perm \
  && bash tools/gpu_profile.sh r03f_prof 2 3 4 \
  && timeout -k 10 300 python tools/bench_handshake.py > gpurun_out/r03f_handshake.jsonl 2>&1
