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
    return L


def main():
    import numpy as np
    import torch
    from tools import synth
    paths = sys.argv[1:]
    n, P, S = 1 << 20, int(os.environ.get("AB_SIZE", 1350)), 0
    S = synth.round_up(P + 32, 128)
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
        libs.append((os.path.basename(p), L, h))

    def seal(L, h):
        assert L.wg_gpu_seal_strided(h, n, P, 0, 0, pt.data_ptr() + 16, S, wire.data_ptr(), S,
                                     st.data_ptr(), stream) == 0

    def open_(L, h):
        assert L.wg_gpu_open_strided(h, n, P + 32, 0, wire.data_ptr(), S, back.data_ptr() + 16, S,
                                     st.data_ptr(), stream) == 0

    ref_wire = None
    for name, L, h in libs:
        wire.zero_(); back.zero_()
        seal(L, h); open_(L, h)
        torch.cuda.synchronize()
        ok = torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P]) and int(st.abs().sum()) == 0
        w = wire.view(n, S)[:, :P + 32]
        if ref_wire is None:
            ref_wire = w.clone()
        same = torch.equal(w, ref_wire)
        print(f"{name}: round-trip {'ok' if ok else 'FAIL'}, wire {'identical' if same else 'DIFFERS'}", flush=True)
    # AB_BURST: back-to-back round trips per variant before each timed one.  The
    # chip is power-capped (tools/power_probe.py): a burst of >= ~0.3 s lets the
    # clock settle to what THIS variant's energy per packet allows.
    burst = int(os.environ.get("AB_BURST", 2))
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
    for name, (s, o) in times.items():
        rt = [a + b for a, b in zip(s, o)]
        print(f"{name:40s} seal med {statistics.median(s):.4f} min {min(s):.4f} | open med "
              f"{statistics.median(o):.4f} min {min(o):.4f} | round trip med {statistics.median(rt):.4f} ms "
              f"= {n * P * 8 / (statistics.median(rt) * 1e-3) / 1e9:.0f} Gbit/s", flush=True)


if __name__ == "__main__":
    main()
