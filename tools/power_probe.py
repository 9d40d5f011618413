#!/usr/bin/env python3
"""Power / clock probe: is the AEAD kernel power-limited?

Runs a long bench.py (seal+open in a loop, config 2) as a child process and
samples `amd-smi metric` (power, clocks, temperature) on the side, then writes
the raw samples and a summary.  Read-only on the GPU (no settings changed).

    python tools/power_probe.py OUT.json [--steps N]
    python tools/power_probe.py OUT.json -- CMD...   (any GPU command, e.g. tools/ab.py on a variant)
"""
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


AMD_SMI = shutil.which("amd-smi") or "/opt/rocm/bin/amd-smi"


def sample(gpu: int = 0):
    """One `amd-smi metric` reading of GPU `gpu` (amd-smi's index), read-only."""
    try:
        # (the interpreter runs the amd-smi script itself: its `#!/usr/bin/env` line is an
        # exec, which a process the profiler's preload initialised for the GPU may not do)
        out = subprocess.run([sys.executable, AMD_SMI, "metric", "-g", str(gpu), "--json"], capture_output=True,
                             text=True, timeout=20)
        return json.loads(out.stdout) if out.returncode == 0 else {"err": out.stderr[-300:]}
    except Exception as e:  # noqa: BLE001
        return {"err": str(e)[:300]}


def summarize(samples):
    """Mean socket power / gfx clock / activity over the samples with gfx activity >= 90 %."""
    rows = []
    for s in samples:
        try:
            g = s["m"]["gpu_data"][0]
            clk = [v["clk"]["value"] for k, v in g["clock"].items() if k.startswith("gfx_")]
            rows.append((g["power"]["socket_power"]["value"], sum(clk) / len(clk),
                         g["usage"]["gfx_activity"]["value"], g["usage"]["umc_activity"]["value"],
                         g.get("throttle", {}).get("ppt_violation_status")))
        except (KeyError, IndexError, TypeError, ZeroDivisionError):
            continue
    busy = [r for r in rows if r[2] >= 90]
    if not busy:
        return {"busy_samples": 0}
    n = len(busy)
    out = {"busy_samples": n, "socket_power_W": round(sum(r[0] for r in busy) / n, 1),
           "gfx_clock_MHz": round(sum(r[1] for r in busy) / n, 1),
           "umc_activity_pct": round(sum(r[3] for r in busy) / n, 1),
           "ppt_violation": sorted({str(r[4]) for r in busy})}
    # the package's energy accumulator between the first and the last busy sample:
    # mean power over that window (not a few instantaneous readings), and the
    # share of it the PPT controller was throttling
    acc = []
    for s in samples:
        try:
            g = s["m"]["gpu_data"][0]
            if g["usage"]["gfx_activity"]["value"] < 90 or "t" not in s:
                continue
            th = g.get("throttle", {})
            acc.append((s["t"], float(g["energy"]["total_energy_consumption"]["value"]),
                        th.get("ppt_accumulated"), th.get("accumulation_counter")))
        except (KeyError, IndexError, TypeError, ValueError):
            continue
    if len(acc) >= 2 and acc[-1][0] > acc[0][0]:
        (t0, e0, p0, c0), (t1, e1, p1, c1) = acc[0], acc[-1]
        out["energy_window_s"] = round(t1 - t0, 3)
        out["socket_power_from_energy_W"] = round((e1 - e0) / (t1 - t0), 1)
        if isinstance(p0, (int, float)) and isinstance(c1, (int, float)) and c1 > c0:
            out["ppt_throttled_fraction"] = round((p1 - p0) / (c1 - c0), 3)
    return out


def main():
    out = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3000
    idle = sample()
    if "--" in sys.argv:
        cmd = sys.argv[sys.argv.index("--") + 1:]
    else:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup", "20",
               "--no-cpu-baseline", "--evp-sample", "0"]
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    samples = []
    t0 = time.time()
    while child.poll() is None:
        s = sample()
        samples.append({"t": round(time.time() - t0, 3), "m": s})
        time.sleep(0.1)
    lines = child.stdout.read().strip().splitlines()
    try:
        bench = json.loads(lines[-1]) if lines else None
    except ValueError:
        bench = {"stdout_tail": lines[-6:]}
    res = {"idle": idle, "samples": samples, "bench": bench, "summary": summarize(samples)}
    with open(out, "w") as f:
        json.dump(res, f)
    print(json.dumps({"summary": res["summary"], "bench": bench})[:3000])


if __name__ == "__main__":
    main()
