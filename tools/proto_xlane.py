#!/usr/bin/env python3
"""Drive tools/proto_xlane.hip (K lanes per packet) against the product seal.

    python tools/proto_xlane.py check  [--size P]           bit-exact vs the product, K = 2, 4, 8
    python tools/proto_xlane.py ab     [--size P] [--rounds R] [--burst B]
                                                            interleaved seal-only bursts, ms per launch
    python tools/proto_xlane.py loop VARIANT [--seconds S]  one variant back to back (for
                                                            tools/power_probe.py: J per launch)

VARIANT: product | k2 | k4 | k8.  Layout: config 2's slots (plaintext at slot + 16,
datagram at slot + 0, stride round_up(P + 32, 128)), one session key, counters =
packet index; 1M x 1350 B or the same payload bytes at other sizes.  The product is
wg_gpu_seal_strided without slot padding (so both write exactly P + 32 bytes per
slot); its bytes are checked against the oracle by tests/test_gpu_parity.py, and a
sample of both against OpenSSL here (tools/evp_check.py).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "build", "proto", "libproto_xlane.so")


def setup(P: int):
    import numpy as np
    import torch

    import neptun_amd
    from tools import synth
    n = (1 << 20) if P == 1350 else max(512, ((1 << 20) * 1350 // P) // 512 * 512)
    S = synth.round_up(P + 32, 128)
    ctx = neptun_amd.GpuContext(0, key_slots=1)
    key = synth.keys(1)
    ctx.set_keys(0, key, np.array([synth.RECEIVER_IDX], np.uint32))
    ctx.set_slot_padding(False)
    pt = synth.device_payloads(n, P, S, "cuda", offset=16)
    lib = ctypes.CDLL(LIB)
    lib.xlane_seal.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p,
                               ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    kb = key[0].tobytes()

    def launch(variant, wire):
        if variant == "product":
            ctx.seal_strided(n, P, 0, 0, pt.data_ptr() + 16, S, wire, S, None, stream)
        else:
            rc = lib.xlane_seal(int(variant[1:]), pt.data_ptr(), S, wire.data_ptr(), S, n, P, kb,
                                synth.RECEIVER_IDX, 0, stream)
            if rc:
                raise RuntimeError(f"xlane_seal rc {rc}")
    return n, S, pt, key, ctx, launch


def check(P: int) -> dict:
    import torch

    from tools import synth
    from tools.evp_check import Evp
    n, S, pt, key, ctx, launch = setup(P)
    ref = torch.full((n * S,), 0xA5, dtype=torch.uint8, device="cuda")
    launch("product", ref)
    torch.cuda.synchronize()
    evp = Evp()
    rows = list(range(0, n, max(1, n // 97))) + [n - 1]
    w = ref.view(n, S)
    p = pt.view(n, S)
    bad_evp = sum(evp.seal_datagram(key[0].tobytes(), synth.RECEIVER_IDX, r, p[r, 16:16 + P].cpu().numpy().tobytes())
                  != w[r, :P + 32].cpu().numpy().tobytes() for r in rows)
    out = {"size": P, "packets": n, "product_vs_openssl_mismatches": bad_evp, "checked_openssl": len(rows)}
    for K in (2, 4, 8):
        wire = torch.full((n * S,), 0xA5, dtype=torch.uint8, device="cuda")
        launch(f"k{K}", wire)
        torch.cuda.synchronize()
        eq = bool(torch.equal(wire, ref))
        out[f"k{K}_bit_exact_vs_product"] = eq
        if not eq:
            diff = (wire.view(n, S) != ref.view(n, S)).any(dim=1).nonzero().flatten()
            out[f"k{K}_bad_packets"] = int(diff.numel())
            out[f"k{K}_first_bad"] = [int(x) for x in diff[:8].cpu()]
        del wire
    ctx.close()
    return out


def ab(P: int, rounds: int, burst: int, variants) -> dict:
    import torch
    n, S, pt, key, ctx, launch = setup(P)
    wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    times = {v: [] for v in variants}
    for v in variants:  # warm
        for _ in range(3):
            launch(v, wire)
    torch.cuda.synchronize()
    for r in range(rounds):
        order = variants if r % 2 == 0 else variants[::-1]
        for v in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(burst):
                launch(v, wire)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / burst)
    ctx.close()
    alg = n * (2 * P + 32)
    return {"size": P, "packets": n, "rounds": rounds, "burst": burst,
            "ms_median": {v: round(statistics.median(t), 4) for v, t in times.items()},
            "ms_min": {v: round(min(t), 4) for v, t in times.items()},
            "hbm_frac_median": {v: round(alg / (statistics.median(t) * 1e-3) / 8e12, 4) for v, t in times.items()}}


def loop(P: int, variant: str, seconds: float) -> dict:
    import torch
    n, S, pt, key, ctx, launch = setup(P)
    wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    for _ in range(5):
        launch(variant, wire)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 0
    t0 = time.time()
    e0.record()
    while time.time() - t0 < seconds:
        for _ in range(50):
            launch(variant, wire)
        k += 50
        torch.cuda.synchronize()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / k
    ctx.close()
    return {"variant": variant, "size": P, "packets": n, "launches": k, "ms_per_launch": round(ms, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("check", "ab", "loop"))
    ap.add_argument("variant", nargs="?", default="product")
    ap.add_argument("--size", type=int, default=1350)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--burst", type=int, default=40)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--variants", default="product,k2,k4,k8")
    a = ap.parse_args()
    if a.mode == "check":
        print(json.dumps(check(a.size)), flush=True)
    elif a.mode == "ab":
        print(json.dumps(ab(a.size, a.rounds, a.burst, a.variants.split(","))), flush=True)
    else:
        print(json.dumps(loop(a.size, a.variant, a.seconds)), flush=True)


if __name__ == "__main__":
    main()
