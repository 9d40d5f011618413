#!/usr/bin/env python3
"""Static per-kernel stats of wg_aead.hip's ISA: scratch (spill) instructions
and VALU instructions in the blocks of loops at depth >= 2 (the round loop of
the persistent kernels) vs outside -- where a spill sits decides what it costs.

    python tools/asm_loop_stats.py [-DWG_FOO=1 ...]
"""
import os
import re
import subprocess
import sys
import tempfile
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "neptun_amd", "csrc")


def asm(defs, src="wg_aead.hip"):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
                        "-I" + os.path.join(ROOT, "include"), *defs, "--cuda-device-only", "-S", src,
                        "-o", out], cwd=CSRC, check=True, capture_output=True)
        return open(out).read()


def stats(text):
    res = {}
    kern, depth = None, 0
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            kern = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            res[kern] = defaultdict(int)
            depth = 0
            continue
        if kern is None:
            continue
        if re.match(r"^(\.LBB|; %bb)", line):
            m = re.search(r"Depth=(\d+)", line)
            depth = int(m.group(1)) if m else 0
            continue
        if line.strip().startswith("s_endpgm"):
            kern = None
            continue
        ins = line.strip().split(" ")[0]
        if not ins or ins.startswith((";", ".")):
            continue
        where = "loop" if depth >= 2 else "outer"
        if ins.startswith("scratch_"):
            res[kern][f"scratch_{where}"] += 1
        if ins.startswith("v_"):
            res[kern][f"valu_{where}"] += 1
    return res


if __name__ == "__main__":
    for k, v in stats(asm(sys.argv[1:])).items():
        if "sync" in k or "text" in k or "strided_kernel<true, false>" in k or "strided_kernel<false, false>" in k:
            print(f"{k[:58]:58s} " + " ".join(f"{a}={v[a]}" for a in sorted(v)))
