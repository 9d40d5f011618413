#!/usr/bin/env python3
"""Host-resident end-to-end rate (north star: "the end-to-end rate including
hipMemcpyAsync to/from pinned host staging must also be measured").

1M x 1350 B packets in pinned host memory (NepTUN slot layout, stride 1408),
sealed and opened through wg_gpu_pipe_* (chunked H2D -> kernel -> D2H over
several streams).  Prints one JSON line per (chunk, depth) and the raw pinned
copy bandwidth for reference.  Not the bench.py metric (that one is
device-resident).
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import neptun_amd
    from tools import synth
    n, P, S = 1 << 20, 1350, 1408
    reps = 5
    ctx = neptun_amd.GpuContext(0, key_slots=1)
    ctx.set_keys(0, synth.keys(1), np.array([synth.RECEIVER_IDX], np.uint32))
    pt = synth.device_payloads(n, P, S, "cuda", offset=16).cpu().pin_memory()
    wire = torch.zeros(n * S, dtype=torch.uint8).pin_memory()
    back = torch.zeros(n * S, dtype=torch.uint8).pin_memory()
    st = torch.zeros(n, dtype=torch.int32).pin_memory()
    # raw pinned copy bandwidth (one direction at a time, one 1.48 GB copy)
    d = torch.empty(n * S, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter(); d.copy_(pt, non_blocking=True); torch.cuda.synchronize()
    h2d = n * S / (time.perf_counter() - t) / 1e9
    t = time.perf_counter(); back.copy_(d, non_blocking=True); torch.cuda.synchronize()
    d2h = n * S / (time.perf_counter() - t) / 1e9
    del d
    print(json.dumps({"pinned_copy_GBps": {"h2d": round(h2d, 2), "d2h": round(d2h, 2)}}), flush=True)
    best = None
    for chunk in (16 << 20, 64 << 20, 256 << 20):
        for depth in (2, 3, 4):
            pipe = neptun_amd.GpuPipe(ctx, chunk_bytes=chunk, depth=depth)
            ts, to = [], []
            for _ in range(reps + 1):
                t0 = time.perf_counter()
                pipe.seal_strided(n, P, 0, 0, pt.data_ptr() + 16, S, wire, S, st)
                t1 = time.perf_counter()
                pipe.open_strided(n, P + 32, 0, wire, S, back.data_ptr() + 16, S, st)
                t2 = time.perf_counter()
                ts.append(t1 - t0); to.append(t2 - t1)
            ts, to = ts[1:], to[1:]
            ok = torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P])
            ms, mo = statistics.median(ts), statistics.median(to)
            line = {"chunk_MiB": chunk >> 20, "depth": depth, "verified": bool(ok),
                    "seal_ms": round(ms * 1e3, 3), "open_ms": round(mo * 1e3, 3),
                    "seal_gbps": round(n * P * 8 / ms / 1e9, 1),
                    "open_gbps": round(n * P * 8 / mo / 1e9, 1),
                    "roundtrip_gbps": round(n * P * 8 / (ms + mo) / 1e9, 1)}
            print(json.dumps(line), flush=True)
            if ok and (best is None or line["roundtrip_gbps"] > best["roundtrip_gbps"]):
                best = line
            pipe.close()
    # a full-duplex tunnel: outbound seal and inbound open batches at the same
    # time, each through its own pipe on its own host thread (ctypes calls drop
    # the GIL), the way a gateway's encrypt and decrypt workers overlap
    import threading
    c = best or {"chunk_MiB": 16, "depth": 3}
    pa = neptun_amd.GpuPipe(ctx, chunk_bytes=c["chunk_MiB"] << 20, depth=c["depth"])
    pb = neptun_amd.GpuPipe(ctx, chunk_bytes=c["chunk_MiB"] << 20, depth=c["depth"])
    wire_in = wire.clone().pin_memory()  # last round's datagrams: the inbound side's input
    st2 = torch.zeros(n, dtype=torch.int32).pin_memory()
    walls = []
    for _ in range(reps + 1):
        back.zero_()
        ta = threading.Thread(target=lambda: pa.seal_strided(n, P, 0, 0, pt.data_ptr() + 16, S, wire, S, st))
        tb = threading.Thread(target=lambda: pb.open_strided(n, P + 32, 0, wire_in, S, back.data_ptr() + 16,
                                                             S, st2))
        t0 = time.perf_counter()
        ta.start(); tb.start(); ta.join(); tb.join()
        walls.append(time.perf_counter() - t0)
    walls = walls[1:]
    ok = torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P]) and \
        torch.equal(wire, wire_in) and int(st.abs().sum()) == 0 and int(st2.abs().sum()) == 0
    mw = statistics.median(walls)
    print(json.dumps({"mode": "full duplex: seal and open batches concurrently (two pipes, two threads)",
                      "chunk_MiB": c["chunk_MiB"], "depth": c["depth"], "verified": bool(ok),
                      "wall_ms": round(mw * 1e3, 3),
                      "each_direction_gbps": round(n * P * 8 / mw / 1e9, 1),
                      "both_directions_gbps": round(2 * n * P * 8 / mw / 1e9, 1)}), flush=True)
    pa.close(); pb.close()
    # zero-copy: the strided kernels address the pinned host buffers directly
    # (torch pin_memory = mapped hipHostMalloc memory), reads and writes share PCIe
    ts, to = [], []
    for _ in range(reps + 1):
        back.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.seal_strided(n, P, 0, 0, pt.data_ptr() + 16, S, wire.data_ptr(), S, st.data_ptr())
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ctx.open_strided(n, P + 32, 0, wire.data_ptr(), S, back.data_ptr() + 16, S, st.data_ptr())
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ts.append(t1 - t0); to.append(t2 - t1)
    ts, to = ts[1:], to[1:]
    ok = torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P]) and int(st.abs().sum()) == 0
    ms, mo = statistics.median(ts), statistics.median(to)
    zc = {"mode": "zero-copy (kernel on pinned host memory)", "verified": bool(ok),
          "seal_ms": round(ms * 1e3, 3), "open_ms": round(mo * 1e3, 3),
          "seal_gbps": round(n * P * 8 / ms / 1e9, 1), "open_gbps": round(n * P * 8 / mo / 1e9, 1),
          "roundtrip_gbps": round(n * P * 8 / (ms + mo) / 1e9, 1)}
    print(json.dumps(zc), flush=True)
    if ok and zc["roundtrip_gbps"] > best["roundtrip_gbps"]:
        best = zc
    print(json.dumps({"best": best, "packets": n, "packet_bytes": P,
                      "note": "host-resident: pinned host in -> GPU -> pinned host out"}), flush=True)


if __name__ == "__main__":
    main()
