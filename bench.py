#!/usr/bin/env python3
"""bench.py -- device-resident ChaCha20-Poly1305 seal+open throughput (BASELINE.json).

One step = one pass of the hot path over one batch: seal 1M x 1350 B packets
(Session::format_packet_data semantics, session.rs:205-259) then open the
resulting 1M datagrams (receive_packet_data, session.rs:265-302), all in HBM
(BASELINE config 2 per GPU; with --gpus 8 it is config 5: 8M packets, 1M per
GPU, contiguous shards, no collective on the data path -> "scaling": "weak").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Rank 0 prints one JSON line.  value = Gbit/s of plaintext round-trip goodput
over all ranks = world * n * P * 8 * K / max_rank(time of K steps).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Gbit/s device-resident ChaCha20-Poly1305 seal+open, 1350B pkts, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=1 << 20, help="packets per GPU")
    ap.add_argument("--size", type=int, default=1350)
    ap.add_argument("--stride", type=int, default=0, help="slot stride (0 = round up to 128)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, affinity)")
    return ap.parse_args()


def cpu_baseline(threads: int) -> dict | None:
    """Config 1 on the host cores: oracle/build/cpu_baseline (NepTUN framing over
    OpenSSL EVP, the stand-in for ring's asm; see oracle/cpu_baseline.c)."""
    exe = os.path.join(ROOT, "oracle", "build", "cpu_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)

    def run(t, reps):
        out = subprocess.run([exe, "--impl", "openssl", "--threads", str(t), "--packets", "65536",
                              "--reps", str(reps)], capture_output=True, text=True, timeout=300)
        if out.returncode:
            raise RuntimeError(out.stderr)
        return json.loads(out.stdout)

    one = run(1, 11)
    many = run(threads, 21)
    return {
        "value": round(many["gbps"], 3),
        "unit": "Gbit/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"config 1: 65536 x 1350 B encap+decap round trip, one session per thread, "
                   f"NepTUN framing (session.rs:205-302) over OpenSSL 3 EVP_chacha20_poly1305 "
                   f"(stand-in for ring 0.17 asm; the Rust reference cannot be built here), "
                   f"median of 21 reps on {threads} threads; 1 thread: {one['gbps']:.3f} Gbit/s"),
        "one_core_gbps": round(one["gbps"], 3),
    }


def load_traffic(kernel: str) -> dict | None:
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None
    return {"bytes_per_launch": k["hbm_bytes_per_launch"], "source": d.get("source", path)}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    import neptun_amd
    from tools import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    n, P = args.packets, args.size
    S = args.stride or synth.round_up(P + 32, 128)
    if S % 16 or S < P + 32:
        raise SystemExit("--stride must be a multiple of 16 and hold P + 32 bytes")
    ctx = neptun_amd.GpuContext(local, key_slots=1)
    key = synth.keys(1)
    ctx.set_keys(0, key, np.array([synth.RECEIVER_IDX], np.uint32))
    # shard: rank r owns packets [r*n, (r+1)*n) of the global batch; counters follow
    counter_base = rank * n
    # NepTUN slot layout (WG_HEADER_OFFSET = 16, device/mod.rs:76): plaintext 16 bytes
    # into each slot, the datagram at the slot start -- both 128-byte-run aligned
    pt = synth.device_payloads(n, P, S, dev, seed=synth.SEED + rank, offset=16)
    wire = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    back = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    st_seal = torch.full((n,), -1, dtype=torch.int32, device=dev)
    st_open = torch.full((n,), -1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step(evs=None):
        if evs is not None:
            evs[0].record(stream)
        ctx.seal_strided(n, P, 0, counter_base, pt.data_ptr() + 16, S, wire, S, st_seal, stream)
        if evs is not None:
            evs[1].record(stream)
        ctx.open_strided(n, P + 32, 0, wire, S, back.data_ptr() + 16, S, st_open, stream)
        if evs is not None:
            evs[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    seal_ms = [e[0].elapsed_time(e[1]) for e in events]
    open_ms = [e[1].elapsed_time(e[2]) for e in events]

    # correctness of what was timed: statuses + round-trip identity (full batch)
    ok = int((st_seal != 0).sum()) == 0 and int((st_open != 0).sum()) == 0
    ok = ok and torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P])
    if world > 1:
        f = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        ok = int(f.item()) == 0
    if not ok:
        print(json.dumps({"error": "round-trip verification failed", "rank": rank}), flush=True)
        sys.exit(1)

    if rank == 0:
        total_pkts = world * n * args.steps
        gbps = total_pkts * P * 8 / elapsed / 1e9
        ms_step = elapsed / args.steps * 1e3
        avg_seal = sum(seal_ms) / len(seal_ms)
        avg_open = sum(open_ms) / len(open_ms)
        # algorithmic HBM bytes per launch: seal reads P, writes P+32; open reads P+32, writes P
        launch_bytes = n * (2 * P + 32)
        dom, dom_ms = ("seal", avg_seal) if avg_seal >= avg_open else ("open", avg_open)
        achieved = launch_bytes / (dom_ms * 1e-3) / 1e9
        kname = "aead_strided_kernel<true>" if dom == "seal" else "aead_strided_kernel<false>"
        tr = load_traffic(kname)
        line = {
            "metric": METRIC,
            "value": round(gbps, 2),
            "unit": "Gbit/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded IPv4/UDP-shaped payloads, one session key, counters = lane index)",
            "config": {
                "workload": f"BASELINE config {'2' if world == 1 else '5'}: {n} x {P} B packets per GPU, "
                            "single session, seal then open, device-resident",
                "packets_per_gpu": n, "packet_bytes": P, "slot_stride": S,
                "global_packets": world * n, "parallelism": f"{world} shard(s), no collective",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": tr["bytes_per_launch"] if tr else None,
                "traffic_source": tr["source"] if tr else None,
                "algorithmic_bytes_per_launch": launch_bytes,
            },
            "kernel_ms": {"seal": round(avg_seal, 4), "open": round(avg_open, 4)},
            "seal_gbps": round(n * P * 8 / (avg_seal * 1e-3) / 1e9, 1),
            "open_gbps": round(n * P * 8 / (avg_open * 1e-3) / 1e9, 1),
            "roundtrip_hbm_frac": round(n * (4 * P + 64) / ((avg_seal + avg_open) * 1e-3) / 1e9
                                        / HBM_PEAK_GBS, 4),
            "verified": "all statuses Ok and open(seal(x)) == x over the whole batch",
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
            try:
                line["cpu_baseline"] = cpu_baseline(threads)
            except Exception as e:  # reported, never fatal to the GPU number
                line["cpu_baseline"] = {"error": str(e)[:200]}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
