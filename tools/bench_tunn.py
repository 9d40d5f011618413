#!/usr/bin/env python3
"""Host-resident rate of the batched Tunn data plane (include/neptun_tunn.h).

One peer pair: Tunn A encapsulates N IPv4 packets of P bytes (host buffers, one
call), Tunn B decapsulates the datagrams (replay window, validation, stats).
This is the drop-in path a NepTUN device would call per batch: host memcpy into
pinned staging, H2D, AEAD kernel, D2H, host copy-out, sequential replay /
truncation pass.  Prints one JSON line per batch size.

    python tools/bench_tunn.py [--sizes 4096,65536] [--P 1350] [--reps 9]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(ph: dict) -> dict:
    """wg_tunn_get_phases averaged per batch call."""
    c = max(1, ph["calls"])
    out = {k: round(v / c, 1) for k, v in ph.items() if k.endswith("_us")}
    out["chunks_per_call"] = round(ph["chunks"] / c, 2)
    return out


def main():
    import numpy as np

    import neptun_amd
    from neptun_amd.tunn import TunnResult, _bind
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,16384,65536")
    ap.add_argument("--P", type=int, default=1350)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--register", action="store_true",
                    help="register the packet buffers (direct, copy-free batches)")
    ap.add_argument("--phase-timing", action="store_true",
                    help="also time the device stages with events (wg_tunn_set_phase_timing)")
    ap.add_argument("--align", type=int, default=-1,
                    help="place every buffer's slot 0 this many bytes past a 4096-byte boundary "
                         "(-1: wherever numpy's allocation lands)")
    a = ap.parse_args()
    P = a.P
    ctx = neptun_amd.GpuContext(0, key_slots=64)
    lib = _bind(ctx._lib)
    ta, tb = neptun_amd.Tunn(ctx, 0), neptun_amd.Tunn(ctx, 16)
    rng = np.random.default_rng(7)
    k1, k2 = rng.integers(0, 256, 32, np.uint8).tobytes(), rng.integers(0, 256, 32, np.uint8).tobytes()
    ta.install_session(21, 34, k2, k1, True)
    tb.install_session(34, 21, k1, k2, True)
    for n in [int(x) for x in a.sizes.split(",")]:
        S = (P + 32 + 63) // 64 * 64
        def place(arr):  # a view of n * S bytes at the requested alignment
            if a.align < 0:
                return arr[:n * S]
            skip = (a.align - arr.ctypes.data) % 4096
            return arr[skip:skip + n * S]
        extra = 8192 if a.align >= 0 else 0
        src_all = rng.integers(0, 256, n * S + extra, np.uint8)
        src = place(src_all)
        v = src.reshape(n, S)
        v[:, 0] = 0x45
        v[:, 2] = P >> 8
        v[:, 3] = P & 255
        wire_all, back_all = np.zeros(n * S + extra, np.uint8), np.zeros(n * S + extra, np.uint8)
        wire, back = place(wire_all), place(back_all)
        offs = np.arange(n, dtype=np.uint64) * S
        src_p = (src.ctypes.data + offs).astype(np.uint64)
        wire_p = (wire.ctypes.data + offs).astype(np.uint64)
        back_p = (back.ctypes.data + offs).astype(np.uint64)
        lens = np.full(n, P, np.uint32)
        wlens = np.full(n, P + 32, np.uint32)
        caps = np.full(n, S, np.uint32)
        if a.register:
            for arr in (src_all, wire_all, back_all):
                ctx.register_host(arr.ctypes.data, arr.nbytes)
        res = (TunnResult * n)()
        vp = ctypes.c_void_p
        te, td = [], []
        # one untimed call each first: staging and batch arrays are allocated there,
        # so the phases below are the steady state's
        assert lib.wg_tunn_encapsulate_batch(ta._h, n, vp(src_p.ctypes.data), vp(lens.ctypes.data),
                                             vp(wire_p.ctypes.data), vp(caps.ctypes.data), res) == 0
        assert lib.wg_tunn_decapsulate_batch(tb._h, n, vp(wire_p.ctypes.data), vp(wlens.ctypes.data),
                                             vp(back_p.ctypes.data), vp(caps.ctypes.data), res) == 0
        for t_ in (ta, tb):
            t_.set_phase_timing(a.phase_timing)
            t_.phases(reset=True)
        for _ in range(a.reps):
            t0 = time.perf_counter()
            rc = lib.wg_tunn_encapsulate_batch(ta._h, n, vp(src_p.ctypes.data), vp(lens.ctypes.data),
                                               vp(wire_p.ctypes.data), vp(caps.ctypes.data), res)
            t1 = time.perf_counter()
            assert rc == 0 and res[0].kind == 2 and res[n - 1].len == P + 32
            rc = lib.wg_tunn_decapsulate_batch(tb._h, n, vp(wire_p.ctypes.data), vp(wlens.ctypes.data),
                                               vp(back_p.ctypes.data), vp(caps.ctypes.data), res)
            t2 = time.perf_counter()
            assert rc == 0 and res[0].kind == 3 and res[n - 1].len == P, (res[0].kind, res[0].status)
            te.append(t1 - t0)
            td.append(t2 - t1)
        ok = bool(np.array_equal(back.reshape(n, S)[:, :P], v[:, :P]))
        ph_e, ph_d = ta.phases(reset=True), tb.phases(reset=True)
        if a.register:
            for arr in (src_all, wire_all, back_all):
                ctx.unregister_host(arr.ctypes.data)
        e, d = statistics.median(te), statistics.median(td)
        print(json.dumps({"packets": n, "P": P, "registered": a.register, "verified": ok,
                          "encap_ms": round(e * 1e3, 3), "decap_ms": round(d * 1e3, 3),
                          "encap_gbps": round(n * P * 8 / e / 1e9, 1),
                          "decap_gbps": round(n * P * 8 / d / 1e9, 1),
                          "roundtrip_gbps": round(n * P * 8 / (e + d) / 1e9, 1),
                          "mpps_roundtrip": round(n / (e + d) / 1e6, 3),
                          "env": {k: v for k, v in os.environ.items() if k.startswith("WG_TUNN_")},
                          "align": a.align if a.align >= 0 else int(wire.ctypes.data % 4096),
                          "phases_encap_per_call_us": per_call(ph_e),
                          "phases_decap_per_call_us": per_call(ph_d)}), flush=True)
    ta.close()
    tb.close()


if __name__ == "__main__":
    main()
