#!/usr/bin/env python3
"""Randomized soak of the batched Tunn's registered-pool (DMA batch) paths against the
sequential Tunn model -- TEST INFRASTRUCTURE (imports oracle/, like tests/).

Each round draws a batch size (1 .. 40,000, skewed small; the early start takes >= 16,384),
a slot size, an output mode (WG_TUNN_DMA_OUT direct / scatter / default), chunk size,
stream form, completion-word policy (WG_TUNN_FLAG) and small-call path (WG_TUNN_SRV),
encapsulates a batch of mostly-1350-byte packets from registered slots and
decapsulates the peer's traffic with replays, too-old counters, tampered tags, forged-
then-real counters, wrong indices and keepalives -- with destination slots on 128-byte
lines, 16 bytes past one, or 8 bytes off 16-byte alignment (each output mode's case) or one dst
outside the registered pool (the rest of the batch takes the staged path).  Results,
every dst byte, replay windows and byte counters must equal the model's.

    python tests/soak_tunn.py SECONDS [SEED]   -> one JSON line per round, then a summary
"""
import json
import os
import random
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle as o  # noqa: E402
from oracle import tunn_model as M  # noqa: E402
from tests.test_tunn_gpu import FIRST_SLOT, SlotArena, check_same, ipv4  # noqa: E402


def main():
    import ctypes

    import numpy as np
    from neptun_amd import GpuContext
    from neptun_amd.tunn import Tunn
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rng = random.Random(seed)
    gpu = GpuContext(0, key_slots=4096)
    t_end = time.time() + secs
    rounds = packets = 0
    while time.time() < t_end:
        n = rng.choice([1, 7, 64, 500, 3000, 12000, 17000, 26000, 40000])
        slot = rng.choice([1408, 1536, 2048])
        # dst slots on 128-byte lines (0), 16 past one (16), or 8 off 16-byte alignment (8):
        # the output modes' alignment cases (direct where the runs sit on lines)
        shift = rng.choice([0, 0, 16, 8])
        env = {"WG_TUNN_DMA_OUT": rng.choice(["direct", "scatter", ""]),
               "WG_TUNN_CHUNK_KB": rng.choice(["", "2048", "8192", "65536"]),
               "WG_TUNN_DMA_STREAMS": rng.choice(["", "0"]),
               "WG_TUNN_SETS": rng.choice(["", "3"]),
               # the kernel's completion word: default (chunks <= 128 packets), never,
               # or every zero-copy latency-form chunk (grids of up to 4096 packets)
               "WG_TUNN_FLAG": rng.choice(["", "0", "4096"]),
               # small calls posted to the engine's resident kernel (round 6, off by default)
               "WG_TUNN_SRV": rng.choice(["", "1"])}
        for k, v in env.items():
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
        stray_at = rng.randrange(n) if rng.random() < 0.2 else -1
        tm, tg = M.Tunn(), Tunn(gpu, FIRST_SLOT)
        local, peer = 3, rng.getrandbits(32)
        rk, sk = rng.randbytes(32), rng.randbytes(32)
        for t in (tm, tg):
            t.set_time(100)
            t.install_session(local, peer, rk, sk, True)
        # outbound
        srcs = [ipv4(rng, 1350 if rng.random() > 0.02 else rng.choice([64, 1349, 700])) for _ in range(n)]
        a_src, a_dst = SlotArena(srcs, slot), SlotArena([], slot + 128, n)
        dptrs = a_dst.ptrs + np.uint64(shift)
        for a in (a_src, a_dst):
            gpu.register_host(*a.window())
        caps = np.full(n, slot, np.uint32)
        dm = [bytearray(b"\xee" * slot) for _ in range(n)]
        res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
        res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, dptrs, caps)
        dg = [bytearray(a_dst.buf[int(a_dst.offs[k]) + shift:int(a_dst.offs[k]) + shift + slot]) for k in range(n)]
        check_same(res_g, res_m, dg, dm, f"soak encap round {rounds}")
        for a in (a_src, a_dst):
            gpu.unregister_host(a.window()[0])
        # inbound: the peer's traffic with damage
        dgs, c = [], 0
        for _ in range(n):
            r = rng.random()
            P = 1350 if rng.random() > 0.02 else rng.choice([0, 64, 1000])
            pt = ipv4(rng, P) if P else b""
            ctr = c if r > 0.03 else max(0, c - rng.randrange(1, 40)) if r > 0.015 else max(0, c - 3000)
            c = max(c, ctr + 1)
            d = bytearray(o.format_packet_data(rk, local, ctr, pt))
            r = rng.random()
            if r < 0.01:
                d[rng.randrange(16, len(d))] ^= 0x04
            elif r < 0.015:
                d[4:8] = struct.pack("<I", local + 8)
            dgs.append(bytes(d))
        for at in range(rng.randrange(1, 200), n - 10, rng.choice([97, 997, 4001])):
            forged = bytearray(dgs[at + 7])
            forged[-1] ^= 0x80
            dgs[at] = bytes(forged)
        a_in, a_out = SlotArena(dgs, slot), SlotArena([], slot + 128, n)
        optrs = a_out.ptrs + np.uint64(shift)
        stray = ctypes.create_string_buffer(b"\xee" * slot, slot)
        if stray_at >= 0:
            optrs[stray_at] = ctypes.addressof(stray)
        for a in (a_in, a_out):
            gpu.register_host(*a.window())
        dm = [bytearray(b"\xee" * slot) for _ in range(n)]
        res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
        res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, optrs, caps)
        dg = [bytearray(a_out.buf[int(a_out.offs[k]) + shift:int(a_out.offs[k]) + shift + slot]) for k in range(n)]
        if stray_at >= 0:
            dg[stray_at] = bytearray(stray.raw)
        check_same(res_g, res_m, dg, dm, f"soak decap round {rounds}")
        assert tg.stats() == (tm.tx_bytes, tm.rx_bytes), rounds
        for a in (a_in, a_out):
            gpu.unregister_host(a.window()[0])
        tg.close()
        rounds += 1
        packets += 2 * n
        print(json.dumps({"round": rounds, "n": n, "slot": slot, "shift": shift, "stray": stray_at >= 0,
                          "env": {k: v for k, v in env.items() if v}}), flush=True)
    print(json.dumps({"summary": True, "seed": seed, "rounds": rounds, "packets": packets, "mismatches": 0}),
          flush=True)
    gpu.close()


if __name__ == "__main__":
    main()
