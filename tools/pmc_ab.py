#!/usr/bin/env python3
"""HBM traffic per launch of variant builds, from rocprofv3 PMC counters over
tools/ab.py (one variant per run; FETCH_SIZE and WRITE_SIZE in separate passes,
never combined with tracing domains; corrections as tools/pmc_traffic.py).

    AB_... env as for tools/ab.py
    python tools/pmc_ab.py OUT.json build/variants/libneptun_gpu_a.so [...]
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.pmc_traffic import short  # noqa: E402


def pmc_pass(counter, outdir, lib):
    import csv
    import glob
    from collections import defaultdict
    d = os.path.join(outdir, counter.lower())
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "tools", "ab.py"), lib]
    env = dict(os.environ, TMPDIR="/tmp", AB_ROUNDS=os.environ.get("AB_ROUNDS", "2"),
               AB_BURST=os.environ.get("AB_BURST", "1"))
    subprocess.run(cmd, check=True, env=env, timeout=300, stdout=subprocess.DEVNULL)
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        acc = defaultdict(float)
        for r in csv.DictReader(open(f)):
            acc[(r["Kernel_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in acc.items():
            vals[k].append(v)
    return vals


def main():
    out, libs = sys.argv[1], sys.argv[2:]
    work = os.path.join(ROOT, "gpurun_out", "pmc_ab", os.path.splitext(os.path.basename(out))[0])
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on tools/ab.py <variant>; "
                     "read = 2*1024*FETCH_SIZE, write = 1024*WRITE_SIZE (tools/pmc_traffic.py)",
           "env": {k: v for k, v in os.environ.items() if k.startswith("AB_")}, "variants": {}}
    for lib in libs:
        name = os.path.basename(lib)
        w = os.path.join(work, name)
        shutil.rmtree(w, ignore_errors=True)
        fetch, write = pmc_pass("FETCH_SIZE", w, lib), pmc_pass("WRITE_SIZE", w, lib)
        ks = {}
        for k in set(fetch) | set(write):
            s = short(k)
            if not s:
                continue
            f = sorted(fetch.get(k, [0.0]))[len(fetch.get(k, [0.0])) // 2]
            wr = sorted(write.get(k, [0.0]))[len(write.get(k, [0.0])) // 2]
            ks[s] = {"hbm_read_bytes": int(f * 2048), "hbm_write_bytes": int(wr * 1024),
                     "dispatches": len(fetch.get(k, []))}
        res["variants"][name] = ks
        print(name, json.dumps(ks), flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
