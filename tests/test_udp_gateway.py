"""The batched Tunn behind real UDP sockets (examples/udp_gateway.c): a
PacketWorkers-shaped driver (packet_workers.rs:178-287) that encapsulates
batches on the GPU and sends them with sendmmsg, receives with recvmmsg and
decapsulates on the GPU, on 127.0.0.1.  64 Ki packets go through; every sent
datagram must equal the sequential model's Tunn::encapsulate output and every
received datagram's TunnResult and destination bytes the model's
Tunn::decapsulate of the same arrival sequence (oracle/tunn_model.py)."""
import json
import os
import random
import struct
import subprocess

import pytest

from oracle import tunn_model as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RES = struct.Struct("<iiIB16s3x")  # wg_tunn_result


def build(tmp_path, cpu=False):
    """cpu: the OpenSSL backend (examples/gw_cpu_tunn.h) -- the same-box CPU line."""
    exe = str(tmp_path / ("udp_gateway_cpu" if cpu else "udp_gateway"))
    lib = os.path.join(ROOT, "neptun_amd")
    extra = ["-DGW_CPU", "-I", os.path.join(ROOT, "examples")] if cpu else []
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-pthread", "-I",
                    os.path.join(ROOT, "include")] + extra + [os.path.join(ROOT, "examples", "udp_gateway.c"),
                    "-L", lib, "-lneptun_gpu", f"-Wl,-rpath,{lib}"] + (["-lcrypto"] if cpu else [])
                   + ["-o", exe], check=True)
    return exe


def ipv4(rng, total):
    b = bytearray(rng.randbytes(total))
    b[0] = 0x45
    b[2:4] = struct.pack(">H", total)
    return bytes(b)


def write_input(path, pkts, a_idx, b_idx, k1, k2):
    with open(path, "wb") as f:
        f.write(b"NGW1" + struct.pack("<III", len(pkts), a_idx, b_idx) + k1 + k2)
        for p in pkts:
            f.write(struct.pack("<I", len(p)) + p)


def read_output(path):
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"NGWO"
    pos = 4
    (n,) = struct.unpack_from("<I", data, pos)
    pos += 4
    sent = []
    for _ in range(n):
        (ln,) = struct.unpack_from("<I", data, pos)
        sent.append(data[pos + 4:pos + 4 + ln])
        pos += 4 + ln
    (nrx,) = struct.unpack_from("<I", data, pos)
    pos += 4
    recv = []
    for _ in range(nrx):
        (ln,) = struct.unpack_from("<I", data, pos)
        dg = data[pos + 4:pos + 4 + ln]
        pos += 4 + ln
        res = RES.unpack_from(data, pos)
        pos += RES.size
        (cap,) = struct.unpack_from("<I", data, pos)
        dst = data[pos + 4:pos + 4 + cap]
        pos += 4 + cap
        recv.append((dg, res, dst))
    return sent, recv


def test_udp_gateway_builds_and_fails_loudly_without_gpu(tmp_path):
    exe = build(tmp_path)
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu-marked test")
    inp = tmp_path / "in.bin"
    write_input(inp, [b"\x45" * 20], 1, 2, bytes(32), bytes(32))
    r = subprocess.run([exe, str(inp), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("pools", ["plain", "reg"])
def test_udp_gateway_64k_packets_match_sequential_tunn(tmp_path, torch_cuda, pools):
    """64 Ki mixed-length packets through the gateway; "reg": its packet pools registered
    (the library's DMA path where a batch's packets form runs, staging elsewhere)."""
    run_and_check(build(tmp_path), tmp_path, 65536, ["reg"] if pools == "reg" else [])


@pytest.mark.parametrize("mode", [("1", []), ("3", ["mux"]), ("4", []), ("5", ["mux=2"])])
def test_udp_gateway_cpu_backend_matches_sequential_tunn(tmp_path, mode):
    """The CPU line (OpenSSL in place of the GPU, same sockets and threads) obeys the
    same sequential-Tunn contract, so the two gateway lines do the same work -- with
    independent pairs, and with "mux" (one encrypt and one decrypt worker whose batches
    mix the pairs: the multi-peer calls)."""
    pairs, extra = mode
    run_and_check(build(tmp_path, cpu=True), tmp_path, 8192, extra, int(pairs))


@pytest.mark.gpu
@pytest.mark.parametrize("pools", ["plain", "reg"])
def test_udp_gateway_mux_multi_peer_batches_match_sequential_tunns(tmp_path, torch_cuda, pools):
    """4 peers behind one encrypt and one decrypt worker: every batch mixes the peers'
    packets (wg_tunn_encapsulate_multi / wg_tunn_decapsulate_multi on the shared engine);
    each peer's datagrams and decapsulated packets equal its own sequential Tunn's."""
    run_and_check(build(tmp_path), tmp_path, 32768, ["mux"] + (["reg"] if pools == "reg" else []), 4)


def run_and_check(exe, tmp_path, n, extra, pairs=1):
    rng = random.Random(61)
    a_idx, b_idx = 0x00C0FE01, 0x00BEEF02
    k1, k2 = rng.randbytes(32), rng.randbytes(32)
    pkts = [ipv4(rng, rng.choice([20, 64, 576, 1350, 1400, rng.randrange(20, 1401)]))
            for _ in range(n)]
    for i in rng.sample(range(len(pkts)), 64):
        pkts[i] = b""  # keepalives
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    write_input(inp, pkts, a_idx, b_idx, k1, k2)
    r = subprocess.run([exe, str(inp), str(out), "1024", str(pairs)] + extra,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    print(summary)
    sent, recv = read_output(out)
    assert summary["lost"] == 0 and len(recv) == len(pkts)
    kinds = set()
    for p in range(pairs):  # pair p: indices + 256 p, its share of the input in order
        lo, hi = n * p // pairs, n * (p + 1) // pairs
        # A: sequential Tunn::encapsulate calls over the pair's packets
        ta = M.Tunn()
        ta.install_session(a_idx + 256 * p, b_idx + 256 * p, k2, k1, True)
        for i in range(lo, hi):
            d = bytearray(len(pkts[i]) + 32)
            kind, st, ln = ta.encapsulate(pkts[i], d)
            assert (kind, st) == (M.WRITE_TO_NETWORK, 0)
            assert sent[i] == bytes(d[:ln]), (p, i)
        # B: Tunn::decapsulate over the pair's arrival sequence
        tb = M.Tunn()
        tb.install_session(b_idx + 256 * p, a_idx + 256 * p, k1, k2, True)
        for j in range(lo, hi):
            dg, res, dst = recv[j]
            d = bytearray(len(dst))
            m = tb.decapsulate(dg, d)
            assert (res[0], res[1], res[2]) == m[:3], (p, j)
            if m[0] == M.WRITE_TO_TUNNEL:
                assert res[3] == m[3] and res[4][:4] == m[4]
            assert dst == bytes(d), (p, j)
            kinds.add(m[0])
    assert kinds == {M.WRITE_TO_TUNNEL, M.DONE}
    # loopback keeps order here, so every IP packet came back as sent
    got = [dst[:res[2]] for dg, res, dst in recv if res[0] == M.WRITE_TO_TUNNEL]
    assert sorted(got) == sorted(p for p in pkts if p)
