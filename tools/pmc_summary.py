#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/gpu.sh step pmc-cmd output) per kernel: mean per dispatch.

Derived numbers (per launch): HBM bytes with the gfx950 corrections of
MI355X_MICROARCH.md "HBM": FETCH_SIZE (KiB) reads half of a wide streaming read
on gfx950 -> x2 (calibrated for our access pattern by tools/probes/microbench_mem*),
WRITE_SIZE (KiB) exact for 16-B/lane stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirpath):
    per = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(dirpath, "p*", "pmc_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        # one row per (dispatch, counter); sum over dimensions first
        acc = defaultdict(float)
        for r in rows:
            key = (r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
        for (k, d, c), v in acc.items():
            per[k][c].append(v)
    return per


def short(name):
    for tag in ("aead_strided_kernel<true>", "aead_strided_kernel<false>", "aead_desc_kernel<true>",
                "aead_desc_kernel<false>"):
        if tag in name:
            return tag
    return name[:60]


def main():
    d = sys.argv[1]
    per = load(d)
    out = {}
    for k, cs in per.items():
        if "wg::" not in k and "kern" not in k and "aead" not in k:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in m:
            m["hbm_read_bytes_x2"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_BUSY_CYCLES" in m and "SQ_WAVE_CYCLES" in m:
            m["valu_active_per_wave_cycle"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        out[short(k)] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
