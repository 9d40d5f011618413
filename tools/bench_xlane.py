"""Small-batch descriptor launches: latency form (wg_xlane.hip, G lanes per packet)
against the throughput forms, per batch size and payload.

    python tools/bench_xlane.py [--sizes 1,50,64,256,1024,4096,16384] [--P 1350] [--reps 200]

For every (n, P) it times R back-to-back seal and open launches on device buffers
(HIP events on the launch stream) with each form -- the default selection, each
forced G, and the throughput forms (lanes = 0) -- and checks that every form's
output equals the throughput form's.  One JSON line per (n, P, form).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,50,64,256,1024,4096,16384")
    ap.add_argument("--P", default="1350")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--forms", default="default,64,32,16,8,off")
    ap.add_argument("--warm-ms", type=float, default=300.0,
                    help="launches before each timed form, to settle the clock (ms)")
    a = ap.parse_args()
    import torch

    import neptun_amd
    from tools import synth

    torch.cuda.set_device(0)
    ctx = neptun_amd.GpuContext(0, key_slots=64)
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 256, (64, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, 64, dtype=np.uint64).astype(np.uint32)
    ctx.set_keys(0, keys, kidx)
    DESC = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("counter", "<u8"), ("len", "<u4"),
                     ("key_slot", "<u4")])
    for P in [int(x) for x in a.P.split(",")]:
        for n in [int(x) for x in a.sizes.split(",")]:
            S = synth.round_up(P + 32, 128)
            src = torch.from_numpy(rng.integers(0, 256, n * S, dtype=np.uint8)).cuda()
            wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
            back = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
            st = torch.zeros(n, dtype=torch.int32, device="cuda")
            d = np.zeros(n, DESC)
            d["src_off"] = np.arange(n) * S + 16
            d["dst_off"] = np.arange(n) * S
            d["counter"] = np.arange(n) + 7
            d["len"] = P
            d["key_slot"] = np.arange(n) % 64
            o = d.copy()
            o["src_off"] = np.arange(n) * S
            o["dst_off"] = np.arange(n) * S + 16
            o["len"] = P + 32
            d_seal = torch.from_numpy(d.view(np.uint8)).cuda()
            d_open = torch.from_numpy(o.view(np.uint8)).cuda()
            ref = None
            for form in a.forms.split(","):
                lanes = {"default": -1, "off": 0}.get(form)
                if lanes is None:
                    lanes = n * int(form)
                ctx.set_xlane_lanes(lanes)
                res = {"n": n, "P": P, "form": form}
                for name, fn, desc, s_in, s_out in (("seal", ctx.seal_batch, d_seal, src, wire),
                                                    ("open", ctx.open_batch, d_open, wire, back)):
                    fn(desc, n, s_in, s_out, st)
                    torch.cuda.synchronize()
                    t_end = time.perf_counter() + a.warm_ms / 1e3
                    while time.perf_counter() < t_end:
                        for _ in range(20):
                            fn(desc, n, s_in, s_out, st)
                        torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.reps):
                        fn(desc, n, s_in, s_out, st)
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / a.reps
                    res[f"{name}_us"] = round(us, 2)
                    res[f"{name}_gbps"] = round(n * P * 8 / us / 1e3, 2)
                    assert int((st != 0).sum()) == 0, f"{name} status"
                out = (wire.clone(), back.clone())
                if ref is None:
                    ref = out
                res["same_as_first"] = bool(torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]))
                res["round_trip_ok"] = bool(torch.equal(back.view(n, S)[:, 16:16 + P], src.view(n, S)[:, 16:16 + P]))
                assert res["same_as_first"] and res["round_trip_ok"], res
                print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
