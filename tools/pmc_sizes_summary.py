#!/usr/bin/env python3
"""Summarise tools/gpu.sh step pmc-sizes: per payload size, the descriptor kernels' HBM
bytes per packet against the algorithmic bytes (seal reads P, writes P + 32; open
the reverse) and against what 32-byte-sector rounding of the packet's own bytes
plus its 32-byte descriptor and 4-byte order entry would give.

    python tools/pmc_sizes_summary.py gpurun_out/TAG > profiles/..._pmc_sizes.json
"""
import glob
import json
import os
import re
import sys


def sectors(lo, hi, g=32):
    return (-(-hi // g) - lo // g) * g


def main():
    d = sys.argv[1]
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc_traffic_size*.json"))):
        P = int(re.search(r"size(\d+)", f).group(1))
        k = json.load(open(f))["kernels"]
        log = open(os.path.join(d, f"pmc_size{P}.log")).read()
        n = None
        m = re.search(r"--per-size (\d+)", log) or re.search(r"per-size (\d+)", json.load(open(f))["source"])
        if m:
            n = int(m.group(1))
        row = {}
        for name, v in k.items():
            seal = name.endswith("<true>")
            alg_r, alg_w = (P, P + 32) if seal else (P + 32, P)
            rd, wr = (16, 16 + P), (0, P + 32)
            if not seal:
                rd, wr = (0, P + 32), (16, 16 + P)
            row["seal" if seal else "open"] = {
                "read_B_per_packet": round(v["hbm_read_bytes"] / n, 1),
                "write_B_per_packet": round(v["hbm_write_bytes"] / n, 1),
                "alg_read": alg_r, "alg_write": alg_w,
                "sector32_read_plus_desc": sectors(*rd) + 36, "sector32_write": sectors(*wr),
                "traffic_over_algorithmic": round(v["hbm_bytes_per_launch"] / (n * (2 * P + 32)), 4)}
        out[P] = {"packets": n, **row}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
