CHECK_DESC="base nofull" bash tools/gpu_r03_check.sh r03f && bash tools/gpu_power_ab.sh r03f/power base perm
