#!/usr/bin/env python3
"""HBM traffic per launch of the bench kernels from rocprofv3 PMC counters.

Runs `bench.py` under rocprofv3 twice -- one pass with FETCH_SIZE, one with
WRITE_SIZE (they do not fit one pass on gfx950; never combined with tracing
domains) -- and applies MI355X_MICROARCH.md "HBM" corrections: FETCH_SIZE is
in KiB and on gfx950 reads half of a wide (16 B/lane) streaming read, so
read bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane
stores, write bytes = 1024 * WRITE_SIZE.  Writes a JSON summary that bench.py
quotes as roofline.traffic.

    python tools/pmc_traffic.py OUT.json [--config N] [bench args...]

bench.py reads profiles/pmc_traffic_config{N}.json (config 2 with --layout neptun:
profiles/pmc_traffic_config2_neptun.json).
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


def pmc_pass(counter, outdir, bench_args):
    d = os.path.join(outdir, counter.lower())
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--sustain-seconds", "0", "--evp-sample", "0"] + bench_args
    subprocess.run(cmd, check=True, env=dict(os.environ, TMPDIR="/tmp"), timeout=600,
                   stdout=subprocess.DEVNULL)
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(float)
        for r in csv.DictReader(open(f)):
            acc[(r["Kernel_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in acc.items():
            vals[k].append(v)
    return vals


def short(name):
    for tag in ("aead_strided_kernel<true, false>", "aead_strided_kernel<false, false>",
                "aead_strided_open_text_kernel",
                "aead_desc_sync_kernel<true>", "aead_desc_sync_kernel<false>",
                "aead_desc_affine_kernel<true>", "aead_desc_affine_kernel<false>",
                "aead_desc_sync_key1_kernel<true>", "aead_desc_sync_key1_kernel<false>",
                "aead_desc_affine_key1_kernel<true>", "aead_desc_affine_key1_kernel<false>",
                "aead_desc_kernel<true>", "aead_desc_kernel<false>"):
        if tag in name:
            return tag
    return None


def main():
    out = sys.argv[1]
    bench_args = sys.argv[2:]
    config = 2
    if "--config" in bench_args:
        config = int(bench_args[bench_args.index("--config") + 1])
    work = os.path.join(ROOT, "gpurun_out", "pmc_traffic", os.path.splitext(os.path.basename(out))[0])
    shutil.rmtree(work, ignore_errors=True)  # no stale CSVs of another config in the globs
    fetch = pmc_pass("FETCH_SIZE", work, bench_args)
    write = pmc_pass("WRITE_SIZE", work, bench_args)
    kernels = {}
    for name in set(fetch) | set(write):
        s = short(name)
        if not s:
            continue
        f = sum(fetch[name]) / len(fetch[name]) if fetch.get(name) else 0.0
        w = sum(write[name]) / len(write[name]) if write.get(name) else 0.0
        kernels[s] = {"fetch_size_kib": f, "write_size_kib": w,
                      "hbm_read_bytes": f * 1024 * 2, "hbm_write_bytes": w * 1024,
                      "hbm_bytes_per_launch": int(f * 1024 * 2 + w * 1024),
                      "dispatches": len(fetch.get(name, []))}
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on bench.py "
                     f"{' '.join(bench_args) or '(config 2)'}; read = 2*1024*FETCH_SIZE (gfx950 "
                     "wide-read correction), write = 1024*WRITE_SIZE",
           "config": config, "kernels": kernels}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
