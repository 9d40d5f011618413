#!/usr/bin/env python3
"""Socket-to-socket rate of the batched Tunn behind UDP (examples/udp_gateway.c):
N x P-byte IPv4 packets through encapsulate (GPU) -> sendmmsg -> 127.0.0.1 ->
recvmmsg -> decapsulate (GPU), for several max_inter_thread_batched_pkts-style
batch sizes (the reference's default is 50, packet_workers.rs:27).

    python tools/bench_gateway.py [N] [P] [batch ...]   -> JSON lines

GW_PAIRS="1 2 4 8" also sweeps the number of independent peers (Tunn pairs,
socket pairs and worker threads) sharing the N packets at each batch size;
GW_REG="0 1" also runs each with the packet pools registered (the DMA path);
GW_MUX="0 1 4" also runs the multi-peer worker shape with that many worker groups ("mux=W":
each group one encrypt and one decrypt worker whose batches mix its pairs, wg_tunn_*_multi); GW_BACKEND="gpu cpu" also runs the CPU line (OpenSSL in place of the GPU Tunn, the
same sockets, threads and batches: examples/gw_cpu_tunn.h).
"""
import json
import os
import random
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.test_udp_gateway import ipv4, write_input  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 1350
    batches = [int(b) for b in sys.argv[3:]] or [50, 256, 1024, 4096]
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(ROOT, "neptun_amd")
        exes = {}
        for backend in os.environ.get("GW_BACKEND", "gpu").split():
            exes[backend] = os.path.join(d, "udp_gateway_" + backend)
            cpu = ["-DGW_CPU", "-I", os.path.join(ROOT, "examples")] if backend == "cpu" else []
            subprocess.run(["gcc", "-O2", "-pthread", "-I", os.path.join(ROOT, "include")] + cpu
                           + [os.path.join(ROOT, "examples", "udp_gateway.c"), "-L", lib, "-lneptun_gpu",
                              f"-Wl,-rpath,{lib}"] + (["-lcrypto"] if cpu else []) + ["-o", exes[backend]],
                           check=True)
        rng = random.Random(7)
        inp = os.path.join(d, "in.bin")
        write_input(inp, [ipv4(rng, P) for _ in range(n)], 11, 22, rng.randbytes(32), rng.randbytes(32))
        pairs = [int(p) for p in os.environ.get("GW_PAIRS", "1").split()]
        regs = [int(x) for x in os.environ.get("GW_REG", "0").split()]
        muxes = [int(x) for x in os.environ.get("GW_MUX", "0").split()]
        runs = [(be, b, p, reg, mx) for b in batches for p in pairs for be in exes for mx in muxes
                for reg in (regs if be == "gpu" else [0])]
        for be, b, p, reg, mx in runs:
            exe = exes[be]
            r = subprocess.run([exe, inp, os.path.join(d, "out.bin"), str(b), str(p)] + (["reg"] if reg else [])
                               + ([f"mux={mx}"] if mx else []),
                               capture_output=True, text=True, timeout=600)
            line = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {
                "error": r.stderr[-300:], "batch": b, "pairs": p, "registered": reg, "backend": be, "mux": mx}
            line["packet_bytes"] = P
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
