#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of wg_aead.hip for a set of -D
flags (hipcc -Rpass-analysis=kernel-resource-usage, device-only, no GPU needed).

    python tools/resource_usage.py [-DWG_FOO=1 ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "neptun_amd", "csrc")


def usage(defs, src="wg_aead.hip"):
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
               "-I" + os.path.join(ROOT, "include"), *defs, "--cuda-device-only", "-S", src,
               "-o", os.path.join(d, "k.s"), "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, cwd=CSRC, capture_output=True, text=True)
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill):\s*(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"kernel": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k.split(" [")[0]] = v
    return rows


if __name__ == "__main__":
    for r in usage(sys.argv[1:]):
        print(f"{r['kernel'][:60]:60s} vgpr {r.get('VGPRs'):>4} vspill {r.get('VGPRs Spill'):>3} "
              f"sspill {r.get('SGPRs Spill'):>4} scratch {r.get('ScratchSize'):>4} occ {r.get('Occupancy')}")
