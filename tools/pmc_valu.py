#!/usr/bin/env python3
"""VALU-side PMC summary of the bench kernels: effective clock, VALU
instructions per wave, VALU-active fraction.  One rocprofv3 pass with
--kernel-trace (durations) and --pmc (never combined with tracing domains).

  clock_GHz        = GRBM_GUI_ACTIVE / 8 (XCDs) / kernel duration
  valu_per_wave    = SQ_INSTS_VALU / SQ_WAVES

(SQ_ACTIVE_INST_VALU is not turned into a "busy fraction": it sums quad-cycles
over co-resident waves, so its quotient by the SIMD cycles can exceed 1.  The
VALU bound is tools/compute_roofline.py: issue floor at this clock vs ms.)
bench.py reads profiles/pmc_valu_config{N}.json.

    python tools/pmc_valu.py OUT.json [bench args...]
    python tools/pmc_valu.py OUT.json --cmd python tools/ab.py build/variants/libX.so
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ["GRBM_GUI_ACTIVE", "SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"]


def short(name):
    for tag in ("aead_strided_kernel<true, false>", "aead_strided_kernel<false, false>",
                "aead_strided_open_text_kernel", "aead_desc_kernel<true>", "aead_desc_kernel<false>",
                "aead_desc_sync_kernel<true>", "aead_desc_sync_kernel<false>",
                "aead_desc_affine_kernel<true>", "aead_desc_affine_kernel<false>",
                "aead_desc_sync_key1_kernel<true>", "aead_desc_sync_key1_kernel<false>",
                "aead_desc_affine_key1_kernel<true>", "aead_desc_affine_key1_kernel<false>"):
        if tag in name:
            return tag
    return None


def main():
    out, bench_args = sys.argv[1], sys.argv[2:]
    d = os.path.join(ROOT, "gpurun_out", "pmc_valu", os.path.splitext(os.path.basename(out))[0])
    shutil.rmtree(d, ignore_errors=True)
    if bench_args[:1] == ["--cmd"]:  # any command, e.g. tools/ab.py on one variant library
        target = bench_args[1:]
    else:
        target = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                  "--no-cpu-baseline", "--sustain-seconds", "0", "--evp-sample", "0"] + bench_args
    cmd = ["rocprofv3", "--kernel-trace", "--pmc", *COUNTERS, "--output-format", "csv", "-d", d,
           "-o", "pmc", "--"] + target
    subprocess.run(cmd, check=True, env=dict(os.environ, TMPDIR="/tmp"), timeout=600,
                   stdout=subprocess.DEVNULL)
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s:
                per[(s, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s:
                dur[(s, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(list)
    for key, c in per.items():
        t = dur.get(key)
        if not t or not c.get("SQ_WAVES"):
            continue
        clk = c["GRBM_GUI_ACTIVE"] / 8 / t
        agg[key[0]].append({
            "ms": t * 1e3, "clock_GHz": clk / 1e9,
            "valu_per_wave": c["SQ_INSTS_VALU"] / c["SQ_WAVES"],
            "salu_per_wave": c["SQ_INSTS_SALU"] / c["SQ_WAVES"],
            "lds_per_wave": c["SQ_INSTS_LDS"] / c["SQ_WAVES"],
            "waves": c["SQ_WAVES"],
        })
    res = {"source": "rocprofv3 --kernel-trace --pmc " + " ".join(COUNTERS) + " on bench.py " +
                     (" ".join(bench_args) or "(config 2)") + " (profiled: clocks read a few % low)",
           "kernels": {k: {m: round(sum(x[m] for x in v) / len(v), 4) for m in v[0]} | {"dispatches": len(v)}
                       for k, v in agg.items()}}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
