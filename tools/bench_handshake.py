#!/usr/bin/env python3
"""Throughput of the batched handshake kernels, one JSON line each:
X25519 operations per second (per-lane scalar and point) and handshake initiations
per second through mac1 + parse_handshake_anon, next to OpenSSL's X25519 on the host
cores (oracle/build/cpu_x25519, 16 threads; the reference's x25519-dalek cannot be
built here).  Inputs are device-resident; every output of the timed run is checked
on a sample against oracle/handshake_model.py."""
import json
import os
import random
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import neptun_amd
    from neptun_amd.gpu import HALF_HANDSHAKE_DTYPE
    from oracle import handshake_model as H
    n = int(os.environ.get("HS_N", 1 << 20))
    ctx = neptun_amd.GpuContext(0, key_slots=1)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    sc = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device="cuda", generator=g)
    pt = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ctx.x25519_batch(n, sc, pt, out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record()
        ctx.x25519_batch(n, sc, pt, out)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    s, p, o = sc.cpu().numpy().tobytes(), pt.cpu().numpy().tobytes(), out.cpu().numpy().tobytes()
    rng = random.Random(2)
    ok = all(o[32 * i:32 * i + 32] == H.x25519(s[32 * i:32 * i + 32], p[32 * i:32 * i + 32])
             for i in rng.sample(range(n), 64))
    t = statistics.median(ts)
    print(json.dumps({"op": "x25519", "n": n, "ms": round(t * 1e3, 3),
                      "ops_per_s": round(n / t, 1), "verified_sample": ok}), flush=True)

    # handshake initiations: 4096 distinct valid messages tiled over the batch
    resp_priv = bytes(range(32))
    resp_pub = H.public_key(resp_priv)
    base = [H.format_handshake_initiation(rng.randbytes(32), resp_pub, rng.randbytes(32), i,
                                          rng.randbytes(12)) for i in range(512)]
    tile = b"".join(base)
    msgs = torch.from_numpy(np.frombuffer(tile * (n // len(base)), np.uint8).copy()).cuda()
    m = n // len(base) * len(base)
    res = torch.zeros(m * HALF_HANDSHAKE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ctx.handshake_anon_batch(resp_priv, m, msgs, 148, res)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record()
        ctx.handshake_anon_batch(resp_priv, m, msgs, 148, res)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    r = res.cpu().numpy().view(HALF_HANDSHAKE_DTYPE)
    ok = bool((r["status"] == 0).all()) and all(
        r[i]["peer_static_public"].tobytes() ==
        H.parse_handshake_anon(resp_priv, resp_pub, base[i % len(base)])[2]
        for i in rng.sample(range(m), 32))
    t = statistics.median(ts)
    print(json.dumps({"op": "handshake_anon (mac1 + parse_handshake_anon)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)
    exe = os.path.join(ROOT, "oracle", "build", "cpu_x25519")
    if os.path.exists(exe):
        threads = min(16, len(os.sched_getaffinity(0)))
        for th in (1, threads):
            r = subprocess.run([exe, "--threads", str(th), "--ops", "20000"], capture_output=True,
                               text=True, timeout=300)
            print(json.dumps({"op": "cpu_baseline x25519 (OpenSSL 3 EVP)", **json.loads(r.stdout)}),
                  flush=True)


if __name__ == "__main__":
    main()
