#!/usr/bin/env python3
"""A/B-time several builds of libneptun_gpu.so in ONE process (interleaved rounds).

    python tools/ab.py build/variants/libneptun_gpu_a.so build/variants/libneptun_gpu_b.so ...

Every variant must produce bit-identical wire bytes and round-trip output; the
first one is the reference.  Prints median/min seal and open ms per variant.
"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bind(path):
    L = ctypes.CDLL(os.path.abspath(path))
    c = ctypes
    vp, u32, u64 = c.c_void_p, c.c_uint32, c.c_uint64
    L.wg_gpu_ctx_create.argtypes = [c.c_int, u32, c.POINTER(vp)]
    L.wg_gpu_set_keys.argtypes = [vp, u32, u32, vp, vp, vp]
    L.wg_gpu_seal_strided.argtypes = [vp, u32, u32, u32, u64, vp, u64, vp, u64, vp, vp]
    L.wg_gpu_open_strided.argtypes = [vp, u32, u32, u32, vp, u64, vp, u64, vp, vp]
    L.wg_gpu_last_error.restype = c.c_char_p
    if hasattr(L, "wg_gpu_ctx_set_slot_padding"):
        L.wg_gpu_ctx_set_slot_padding.argtypes = [vp, c.c_int]
    for fn in (L.wg_gpu_seal_batch, L.wg_gpu_open_batch):
        fn.argtypes = [vp, vp, u32, vp, vp, vp, vp]
    for fn in (L.wg_gpu_seal_batch_ordered, L.wg_gpu_open_batch_ordered):
        fn.argtypes = [vp, vp, vp, u32, vp, vp, vp, vp]
    L.wg_gpu_plan_batch.argtypes = [vp, c.c_int, vp, u32, vp, vp, vp]
    return L


def main_desc(paths, cfg):
    """AB_CONFIG=3|4: the descriptor kernels on BASELINE config 3 / 4 batches
    (AB_PEERS x AB_PER_PEER for config 4, AB_PER_SIZE per size for config 3)."""
    import numpy as np
    import torch
    from tools import synth, workloads
    dev = torch.device("cuda", 0)
    if cfg == 3:
        b = workloads.config3(int(os.environ.get("AB_PER_SIZE", 1 << 18)), dev)
        nkeys = 1
    else:
        peers = int(os.environ.get("AB_PEERS", 4096))
        b = workloads.config4(peers, int(os.environ.get("AB_PER_PEER", 1024)), 1350, dev)
        nkeys = peers
    keys = synth.keys(nkeys)
    idx = np.full(nkeys, synth.RECEIVER_IDX, np.uint32) + np.arange(nkeys, dtype=np.uint32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = []
    for p in paths:
        L = bind(p)
        h = ctypes.c_void_p()
        assert L.wg_gpu_ctx_create(0, nkeys, ctypes.byref(h)) == 0, L.wg_gpu_last_error()
        assert L.wg_gpu_set_keys(h, 0, nkeys, keys.ctypes.data, idx.ctypes.data, stream) == 0
        libs.append((os.path.basename(p), L, h))

    def seal(L, h):
        if cfg == 3:
            assert L.wg_gpu_plan_batch(h, 1, b.d_seal.data_ptr(), b.n, b.order.data_ptr(),
                                       b.scratch.data_ptr(), stream) == 0
            assert L.wg_gpu_seal_batch_ordered(h, b.d_seal.data_ptr(), b.order.data_ptr(), b.n,
                                               b.pt.data_ptr(), b.wire.data_ptr(),
                                               b.st_seal.data_ptr(), stream) == 0
        else:
            assert L.wg_gpu_seal_batch(h, b.d_seal.data_ptr(), b.n, b.pt.data_ptr(), b.wire.data_ptr(),
                                       b.st_seal.data_ptr(), stream) == 0

    def open_(L, h):
        if cfg == 3:
            assert L.wg_gpu_open_batch_ordered(h, b.d_open.data_ptr(), b.order.data_ptr(), b.n,
                                               b.wire.data_ptr(), b.out.data_ptr(),
                                               b.st_open.data_ptr(), stream) == 0
        else:
            assert L.wg_gpu_open_batch(h, b.d_open.data_ptr(), b.n, b.wire.data_ptr(), b.out.data_ptr(),
                                       b.st_open.data_ptr(), stream) == 0

    ref = None
    for name, L, h in libs:
        b.wire.zero_(); b.out.zero_()
        seal(L, h); open_(L, h)
        torch.cuda.synchronize()
        ok = int((b.st_seal != 0).sum()) == 0 and int((b.st_open != 0).sum()) == 0 and b.round_trip_equal()
        if ref is None:
            ref = b.wire.clone()
        print(f"{name}: round-trip {'ok' if ok else 'FAIL'}, wire "
              f"{'identical' if torch.equal(b.wire, ref) else 'DIFFERS'}", flush=True)
    burst = int(os.environ.get("AB_BURST", 2))
    rounds = int(os.environ.get("AB_ROUNDS", 10))
    times = {name: ([], []) for name, _, _ in libs}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(rounds):
        for name, L, h in libs:
            for _ in range(burst):
                seal(L, h); open_(L, h)
            ev[0].record(); seal(L, h); ev[1].record(); open_(L, h); ev[2].record()
            torch.cuda.synchronize()
            times[name][0].append(ev[0].elapsed_time(ev[1]))
            times[name][1].append(ev[1].elapsed_time(ev[2]))
    pay = float(b.sizes.astype(np.int64).sum())
    for name, (s_, o_) in times.items():
        rt = [a + c for a, c in zip(s_, o_)]
        print(f"{name:40s} config {cfg}: seal med {statistics.median(s_):.4f} | open med "
              f"{statistics.median(o_):.4f} | round trip {statistics.median(rt):.4f} ms = "
              f"{pay * 8 / (statistics.median(rt) * 1e-3) / 1e9:.0f} Gbit/s", flush=True)


def main():
    import numpy as np
    import torch
    from tools import synth
    paths = sys.argv[1:]
    if os.environ.get("AB_CONFIG", "2") != "2":
        return main_desc(paths, int(os.environ["AB_CONFIG"]))
    n, P, S = int(os.environ.get("AB_N", 1 << 20)), int(os.environ.get("AB_SIZE", 1350)), 0
    oo = int(os.environ.get("AB_OPEN_OFF", 16))  # open's plaintext offset in its output slot
    wo = int(os.environ.get("AB_WIRE_OFF", 0))   # seal's datagram offset in its wire slot
    S = int(os.environ.get("AB_STRIDE", 0)) or synth.round_up(P + 32, 128)
    rounds = int(os.environ.get("AB_ROUNDS", 15))
    dev = torch.device("cuda", 0)
    pt = synth.device_payloads(n, P, S, dev, offset=16)
    wire = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    back = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    key = synth.keys(1)
    idx = np.array([synth.RECEIVER_IDX], np.uint32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = []
    for p in paths:
        L = bind(p)
        h = ctypes.c_void_p()
        assert L.wg_gpu_ctx_create(0, 1, ctypes.byref(h)) == 0, L.wg_gpu_last_error()
        assert L.wg_gpu_set_keys(h, 0, 1, key.ctypes.data, idx.ctypes.data, stream) == 0
        if os.environ.get("AB_PAD"):  # slot padding (wg_gpu_ctx_set_slot_padding)
            assert L.wg_gpu_ctx_set_slot_padding(h, int(os.environ["AB_PAD"])) == 0
        libs.append((os.path.basename(p), L, h))

    def seal(L, h):
        assert L.wg_gpu_seal_strided(h, n, P, 0, 0, pt.data_ptr() + 16, S, wire.data_ptr() + wo, S,
                                     st.data_ptr(), stream) == 0

    def open_(L, h):
        assert L.wg_gpu_open_strided(h, n, P + 32, 0, wire.data_ptr() + wo, S, back.data_ptr() + oo, S,
                                     st.data_ptr(), stream) == 0

    ref_wire = None
    for name, L, h in libs:
        wire.zero_(); back.zero_()
        seal(L, h); open_(L, h)
        torch.cuda.synchronize()
        ok = torch.equal(back.view(n, S)[:, oo:oo + P], pt.view(n, S)[:, 16:16 + P]) and int(st.abs().sum()) == 0
        w = wire.view(n, S)[:, wo:wo + P + 32]
        if ref_wire is None:
            ref_wire = w.clone()
        same = torch.equal(w, ref_wire)
        print(f"{name}: round-trip {'ok' if ok else 'FAIL'}, wire {'identical' if same else 'DIFFERS'}", flush=True)
    # AB_BURST: back-to-back round trips per variant before each timed one.  The
    # chip is power-capped (tools/power_probe.py): a burst of >= ~0.3 s lets the
    # clock settle to what THIS variant's energy per packet allows.
    burst = int(os.environ.get("AB_BURST", 2))
    # AB_SEAL_ONLY: bursts of seals only (timing ablations whose open fails and
    # zero-fills would otherwise set a different power state for the next seal)
    seal_only = bool(os.environ.get("AB_SEAL_ONLY"))
    times = {name: ([], []) for name, _, _ in libs}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(rounds):
        for name, L, h in libs:
            for _ in range(burst):
                seal(L, h)
                if not seal_only:
                    open_(L, h)
            ev[0].record(); seal(L, h); ev[1].record()
            if seal_only:
                seal(L, h)
            else:
                open_(L, h)
            ev[2].record()
            torch.cuda.synchronize()
            times[name][0].append(ev[0].elapsed_time(ev[1]))
            times[name][1].append(ev[1].elapsed_time(ev[2]))
    for name, (s, o) in times.items():
        rt = [a + b for a, b in zip(s, o)]
        print(f"{name:40s} seal med {statistics.median(s):.4f} min {min(s):.4f} | open med "
              f"{statistics.median(o):.4f} min {min(o):.4f} | round trip med {statistics.median(rt):.4f} ms "
              f"= {n * P * 8 / (statistics.median(rt) * 1e-3) / 1e9:.0f} Gbit/s", flush=True)


if __name__ == "__main__":
    main()
