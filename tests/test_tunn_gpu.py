"""Batched Tunn (neptun_amd/csrc/wg_tunn.cpp, AEAD on the GPU) == N sequential
calls of the Tunn data plane (oracle/tunn_model.py, restating mod.rs:295-380,
545-670 and session.rs:40-302): same TunnResult per packet, same bytes in
every destination buffer, same counters, replay windows and byte stats.

Traffic covers what the reference's tests and code paths distinguish:
in-order, reordered, duplicated and too-old counters (session.rs:367-414),
tampered tags, wrong receiver index, unknown session, handshake-shaped and
malformed datagrams, keepalives, IPv4/IPv6 packets with valid and truncated
length fields, undersized destination buffers, and a session switch.
"""
import random
import struct

import pytest

from oracle import tunn_model as M
from oracle import pyoracle as o

pytestmark = pytest.mark.gpu

FIRST_SLOT = 4000  # the session fixture's context has 4096 slots


def ipv4(rng, total, claimed=None):
    b = bytearray(rng.randbytes(total))
    b[0] = 0x45
    b[2:4] = struct.pack(">H", total if claimed is None else claimed)
    return bytes(b)


def ipv6(rng, total, claimed=None):
    b = bytearray(rng.randbytes(total))
    b[0] = 0x60
    b[4:6] = struct.pack(">H", (total - 40) if claimed is None else claimed)
    return bytes(b)


def plaintexts(rng, n):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.45:
            out.append(ipv4(rng, rng.choice([20, 64, 576, 1350, rng.randrange(20, 1500)])))
        elif r < 0.7:
            out.append(ipv6(rng, rng.choice([40, 96, 1280, rng.randrange(40, 1500)])))
        elif r < 0.75:
            out.append(b"")  # keepalive
        elif r < 0.8:
            t = rng.randrange(24, 200)
            out.append(ipv4(rng, t, claimed=t + rng.randrange(1, 50)))  # truncated
        elif r < 0.85:
            out.append(ipv6(rng, 60, claimed=100))
        elif r < 0.9:
            b = bytearray(rng.randbytes(rng.randrange(1, 60)))
            b[0] = 0x75  # neither v4 nor v6
            out.append(bytes(b))
        elif r < 0.95:
            out.append(ipv4(rng, 200, claimed=100))  # padded: len = claimed
        else:
            out.append(bytes([0x45]) + rng.randbytes(rng.randrange(0, 19)))  # v4 nibble, < 20 B
    return out


def make_pair(gpu, rng):
    tm, tg = M.Tunn(), None
    from neptun_amd.tunn import Tunn
    tg = Tunn(gpu, FIRST_SLOT)
    sessions = []
    for j, local in enumerate((3, 12)):  # ring slots 3 and 4, established at t = 100, 200
        rk, sk = rng.randbytes(32), rng.randbytes(32)
        peer = rng.getrandbits(32)
        for t in (tm, tg):
            t.set_time(100 * (j + 1))
            t.install_session(local, peer, rk, sk, True)
        sessions.append((local, peer, rk, sk))
    return tm, tg, sessions


def check_same(res_g, res_m, dst_g, dst_m, what):
    assert len(res_g) == len(res_m)
    for i, (g, m) in enumerate(zip(res_g, res_m)):
        kind, st, ln = m[:3]
        assert (g[0], g[1], g[2]) == (kind, st, ln), (what, i, g[:3], m[:3])
        if len(m) > 3 and kind == M.WRITE_TO_TUNNEL:
            v, ip = m[3], m[4]
            assert g[3] == v and g[4][:len(ip)] == ip, (what, i)
        assert bytes(dst_g[i]) == bytes(dst_m[i]), (what, i)


def datagrams(rng, sessions, n, ctr_state):
    """Peer-side traffic for the sessions plus damaged / foreign messages."""
    out = []
    pts = plaintexts(rng, n)
    for j in range(n):
        local, peer, rk, sk = sessions[rng.randrange(len(sessions))]
        r = rng.random()
        c = ctr_state.setdefault(local, 0)
        if r < 0.55:
            ctr = c
            ctr_state[local] = c + 1
        elif r < 0.7:
            ctr = max(0, c - rng.randrange(1, 100))  # reorder / duplicate inside the window
        elif r < 0.73:
            ctr = max(0, c - rng.randrange(1100, 5000))  # older than the window
        elif r < 0.76:
            ctr = c + rng.randrange(2, 2500)  # loss burst / jump past the window
            ctr_state[local] = ctr + 1
        else:
            ctr = c
            ctr_state[local] = c + 1
        d = bytearray(o.format_packet_data(rk, local, ctr, pts[j]))
        r = rng.random()
        if r < 0.04:
            d[rng.randrange(16, len(d))] ^= 1 << rng.randrange(8)  # tamper ct or tag
        elif r < 0.06:
            d[4:8] = struct.pack("<I", local + 8)  # same ring slot, wrong index
        elif r < 0.08:
            d[4:8] = struct.pack("<I", 6)  # ring slot with no session
        elif r < 0.09:
            d = bytearray(struct.pack("<I", 1) + rng.randbytes(144))  # handshake init
        elif r < 0.10:
            d = bytearray(struct.pack("<I", 2) + rng.randbytes(88))  # handshake response
        elif r < 0.11:
            d = bytearray(struct.pack("<I", 3) + rng.randbytes(60))  # cookie reply
        elif r < 0.12:
            d = bytearray(rng.randbytes(rng.randrange(0, 4)))  # empty / too short
        elif r < 0.13:
            d = d[:rng.randrange(4, 32)]  # truncated data message
        elif r < 0.14:
            d[0] = 7  # unknown type
        out.append(bytes(d))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_decapsulate_batch_matches_sequential_tunn(gpu, seed):
    rng = random.Random(seed)
    tm, tg, sessions = make_pair(gpu, rng)
    ctr_state = {}
    for batch in range(4):
        dgs = datagrams(rng, sessions, 600, ctr_state)
        caps = []
        for d in dgs:
            need = max(len(d) - 16, 0)
            caps.append(need if rng.random() > 0.03 else max(need - rng.randrange(1, 17), 0))
        dst_m = [bytearray(b"\xee" * c) for c in caps]
        dst_g = [bytearray(b"\xee" * c) for c in caps]
        res_m = [tm.decapsulate(d, dm) for d, dm in zip(dgs, dst_m)]
        res_g = tg.decapsulate_batch(dgs, dst_g)
        check_same(res_g, res_m, dst_g, dst_m, f"decap batch {batch}")
        kinds = {r[0] for r in res_m}
        assert {M.WRITE_TO_TUNNEL, M.ERR}.issubset(kinds)
    for local, *_ in sessions:
        ctr, w = tg.session_counters(local % M.N_SESSIONS)
        sm = tm.sessions[local % M.N_SESSIONS]
        assert w.next == sm.window.next and list(w.bitmap) == sm.window.bitmap
        assert w.receive_cnt == sm.window.receive_cnt
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()


@pytest.mark.parametrize("seed", [4, 5])
def test_encapsulate_batch_matches_sequential_tunn(gpu, seed):
    rng = random.Random(seed)
    tm, tg, sessions = make_pair(gpu, rng)
    for batch in range(3):
        srcs = [rng.randbytes(rng.choice([0, 1, 15, 16, 17, 64, 1350, rng.randrange(0, 9000)]))
                for _ in range(500)]
        caps = []
        for s in srcs:
            r = rng.random()
            caps.append(len(s) + 32 + rng.randrange(0, 40) if r > 0.06 else
                        len(s) + 16 + rng.randrange(0, 16) if r > 0.03 else len(s) + rng.randrange(0, 16))
        dst_m = [bytearray(b"\xee" * c) for c in caps]
        dst_g = [bytearray(b"\xee" * c) for c in caps]
        res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dst_m)]
        res_g = tg.encapsulate_batch(srcs, dst_g)
        check_same(res_g, res_m, dst_g, dst_m, f"encap batch {batch}")
        # the peer receives what we sent: a keepalive / arbitrary payload path through decap
        if batch == 1:
            # switch current session: a valid packet on the first session (older session
            # timer) must not take over from the newer one (set_current_session, mod.rs:528-542)
            local, peer, rk, sk = sessions[0]
            d = o.format_packet_data(rk, local, 0, b"")
            dm, dg = bytearray(16), bytearray(16)
            check_same(tg.decapsulate_batch([d], [dg]), [tm.decapsulate(d, dm)], [dg], [dm], "ka")
            assert tm.current == sessions[1][0]
    for local, *_ in sessions:
        ctr, _ = tg.session_counters(local % M.N_SESSIONS)
        assert ctr == tm.sessions[local % M.N_SESSIONS].sending_counter
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()


def test_round_trip_between_two_tunns(gpu):
    """Two GPU Tunns as peers: A encapsulates, B decapsulates to the same IP packets."""
    from neptun_amd.tunn import Tunn
    rng = random.Random(9)
    a, b = Tunn(gpu, FIRST_SLOT), Tunn(gpu, FIRST_SLOT - 16)
    k1, k2 = rng.randbytes(32), rng.randbytes(32)
    a.install_session(21, 34, k2, k1, True)  # a sends with k1 to index 34
    b.install_session(34, 21, k1, k2, True)
    pkts = [ipv4(rng, rng.randrange(20, 1500)) for _ in range(300)]
    wires = [bytearray(len(p) + 32) for p in pkts]
    res = a.encapsulate_batch(pkts, wires)
    assert all(r[0] == M.WRITE_TO_NETWORK for r in res)
    outs = [bytearray(len(p) + 16) for p in pkts]
    res = b.decapsulate_batch([bytes(w) for w in wires], outs)
    assert all(r[0] == M.WRITE_TO_TUNNEL for r in res)
    assert all(bytes(o_[:len(p)]) == p for o_, p in zip(outs, pkts))
    # replaying the whole batch is refused packet by packet
    res = b.decapsulate_batch([bytes(w) for w in wires], outs)
    assert all(r[:2] == (M.ERR, M.DUPLICATE_COUNTER) for r in res)
    a.close()
    b.close()


def test_no_session_and_argument_errors(gpu):
    """encapsulate without a session -> NOT_DATA (the CPU Tunn handshakes and queues,
    mod.rs:325-337); the src copy into dst[16..] happens first, like the reference."""
    from neptun_amd.tunn import Tunn
    tm, tg = M.Tunn(), Tunn(gpu, FIRST_SLOT)
    srcs = [b"\x45" * 40, b"", b"abc" * 10]
    caps = [100, 32, 20]
    dm = [bytearray(b"\xee" * c) for c in caps]
    dg = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
    check_same(tg.encapsulate_batch(srcs, dg), res_m, dg, dm, "no session")
    assert [r[:2] for r in res_m] == [(M.NOT_DATA, M.NO_CURRENT_SESSION)] * 2 + [(M.ERR, M.INVALID_LENGTH)]
    tg.close()


@pytest.mark.parametrize("seed", [7, 8])
def test_decrypt_batch_matches_xray_decrypt(gpu, seed):
    """Tunn::decrypt (xray, mod.rs:383-417): either direction's key, no replay window --
    so duplicates decrypt again; keepalives are UnexpectedPacket."""
    rng = random.Random(seed)
    tm, tg, sessions = make_pair(gpu, rng)
    dgs = datagrams(rng, sessions, 500, {})
    # our own outbound traffic (receiver_idx = peer index, sending key) and its duplicates
    for local, peer, rk, sk in sessions:
        for c, p in enumerate(plaintexts(rng, 60)):
            dgs.append(o.format_packet_data(sk, peer, c % 40, p))
    rng.shuffle(dgs)
    caps = [max(len(d) - 16, 0) if rng.random() > 0.03 else max(len(d) - 20, 0) for d in dgs]
    dm = [bytearray(b"\xee" * c) for c in caps]
    dg = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.decrypt(d, x) for d, x in zip(dgs, dm)]
    check_same(tg.decrypt_batch(dgs, dg), res_m, dg, dm, "decrypt")
    codes = {r[:2] for r in res_m}
    assert (M.ERR, M.UNEXPECTED_PACKET) in codes and (M.ERR, M.WRONG_PACKET_TYPE) in codes
    assert sum(r[0] == M.WRITE_TO_TUNNEL for r in res_m) > 300
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()


def test_multi_chunk_pipeline_matches_sequential_tunn(gpu, monkeypatch):
    """Batches of ~12 MB run as several 4 MiB chunks through the double-buffered
    staging pipeline; results must not depend on the chunking (counters across
    chunk edges, replay decisions in packet order across chunks)."""
    monkeypatch.setenv("WG_TUNN_CHUNK_KB", "4096")
    rng = random.Random(77)
    tm, tg, sessions = make_pair(gpu, rng)
    srcs = [ipv4(rng, rng.choice([1350, 1400, rng.randrange(20, 1500)])) for _ in range(9000)]
    caps = [len(s) + 32 for s in srcs]
    dm = [bytearray(c) for c in caps]
    dg = [bytearray(c) for c in caps]
    res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
    check_same(tg.encapsulate_batch(srcs, dg), res_m, dg, dm, "encap multi-chunk")
    dgs = datagrams(rng, sessions, 9000, {})
    caps = [max(len(d) - 16, 0) for d in dgs]
    dm = [bytearray(b"\xee" * c) for c in caps]
    dg = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
    check_same(tg.decapsulate_batch(dgs, dg), res_m, dg, dm, "decap multi-chunk")
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()


def test_session_timers_pick_the_current_session(gpu):
    """set_current_session compares timers.session_timers (mod.rs:528-542), not the
    install order: a session installed LATER but with an OLDER session timer does
    not take over, and traffic on it does not switch the sending session."""
    from neptun_amd.tunn import Tunn
    rng = random.Random(31)
    tm, tg = M.Tunn(), Tunn(gpu, FIRST_SLOT)
    keys = {loc: (rng.randbytes(32), rng.randbytes(32), rng.getrandbits(32)) for loc in (9, 18, 27)}
    for loc, now in ((9, 200), (18, 100), (27, 300)):
        rk, sk, peer = keys[loc]
        for t in (tm, tg):
            t.set_time(now)
            t.install_session(loc, peer, rk, sk, True)
        if loc == 18:  # installed after 9, but its timer is older: 9 stays current
            assert tm.current == 9
    assert tm.current == 27
    # data on the older sessions must not move the sending session off 27
    for loc in (9, 18):
        rk, sk, peer = keys[loc]
        d = o.format_packet_data(rk, loc, 0, b"")
        dm, dg = bytearray(16), bytearray(16)
        check_same(tg.decapsulate_batch([d], [dg]), [tm.decapsulate(d, dm)], [dg], [dm], "ka")
    assert tm.current == 27
    srcs = [ipv4(rng, 100) for _ in range(3)]
    dm = [bytearray(132) for _ in srcs]
    dg = [bytearray(132) for _ in srcs]
    res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
    check_same(tg.encapsulate_batch(srcs, dg), res_m, dg, dm, "encap on the current session")
    assert all(struct.unpack_from("<I", bytes(d), 4)[0] == keys[27][2] for d in dg)
    tg.close()


def test_failed_batch_leaves_the_pipeline_clean(gpu, monkeypatch):
    """A batch that fails part-way (injected HIP error after chunk 1 of 5) drains both
    staging sets; its selected packets read as failed; the next batch runs normally
    and equals the model (counters the failed batch reserved stay consumed)."""
    from neptun_amd import NeptunGpuError
    rng = random.Random(41)
    tm, tg, sessions = make_pair(gpu, rng)
    monkeypatch.setenv("WG_TUNN_CHUNK_KB", "1024")
    srcs = [ipv4(rng, 1350) for _ in range(3500)]  # ~5 MB: 5 chunks of 1 MiB
    dg = [bytearray(1382) for _ in srcs]
    monkeypatch.setenv("WG_TUNN_FAIL_CHUNK", "1")
    with pytest.raises(NeptunGpuError):
        tg.encapsulate_batch(srcs, dg)
    monkeypatch.delenv("WG_TUNN_FAIL_CHUNK")
    tm.sessions[tm.current % M.N_SESSIONS].sending_counter += len(srcs)  # reserved by the failed call
    for batch in range(2):
        srcs = [ipv4(rng, rng.choice([64, 1350, rng.randrange(20, 1500)])) for _ in range(3500)]
        caps = [len(s) + 32 for s in srcs]
        dm = [bytearray(c) for c in caps]
        dg = [bytearray(c) for c in caps]
        res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
        check_same(tg.encapsulate_batch(srcs, dg), res_m, dg, dm, f"after failure {batch}")
    # a decapsulate batch that fails before its first chunk is unpacked leaves the
    # replay windows untouched; the next batch equals the model
    dgs = datagrams(rng, sessions, 3500, {})
    monkeypatch.setenv("WG_TUNN_FAIL_CHUNK", "0")
    with pytest.raises(NeptunGpuError):
        tg.decapsulate_batch(dgs, [bytearray(max(len(d) - 16, 0)) for d in dgs])
    monkeypatch.delenv("WG_TUNN_FAIL_CHUNK")
    caps = [max(len(d) - 16, 0) for d in dgs]
    dm = [bytearray(b"\xee" * c) for c in caps]
    dg = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
    check_same(tg.decapsulate_batch(dgs, dg), res_m, dg, dm, "decap after failure")
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()


class Arena:
    """Packets laid out in one numpy buffer (16-byte aligned slots) so it can be
    registered with the Tunn for direct, copy-free batches."""

    def __init__(self, blobs, caps, fill=0xEE):
        import numpy as np
        self.caps = [max(c, 1) for c in caps]
        slot = [(max(len(b), c) + 64 + 15) // 16 * 16 for b, c in zip(blobs, self.caps)]
        self.offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.uint64)
        self.buf = np.full(int(sum(slot)) + 4096, fill, np.uint8)
        base = self.buf.ctypes.data
        self.pad = (-base) % 4096  # page-align the registered window
        self.offs += self.pad
        for o, b in zip(self.offs, blobs):
            self.buf[int(o):int(o) + len(b)] = np.frombuffer(b, np.uint8)
        self.ptrs = (base + self.offs).astype(np.uint64)
        self.lens = np.array([len(b) for b in blobs], np.uint32)

    def window(self):
        return self.buf.ctypes.data + self.pad, len(self.buf) - self.pad

    def get(self, k, n):
        o = int(self.offs[k])
        return bytes(self.buf[o:o + n])


@pytest.mark.parametrize("seed", [21, 22])
def test_registered_direct_batches_match_sequential_tunn(gpu, seed):
    """Caller buffers registered with wg_tunn_register_host: encapsulate reads and
    writes them directly, decapsulate / decrypt read datagrams directly; results,
    destination bytes and state equal the sequential model's."""
    import numpy as np
    rng = random.Random(seed)
    tm, tg, sessions = make_pair(gpu, rng)
    srcs = [ipv4(rng, rng.choice([20, 64, 1350, rng.randrange(20, 1500)])) for _ in range(3000)]
    caps = [len(s) + 32 + rng.randrange(0, 3) * 16 for s in srcs]
    a_src = Arena(srcs, [0] * len(srcs))
    a_dst = Arena([b""] * len(srcs), caps)
    for a in (a_src, a_dst):
        gpu.register_host(*a.window())
    dm = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
    res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, a_dst.ptrs, np.array(caps, np.uint32))
    dg = [bytearray(a_dst.get(k, caps[k])) for k in range(len(srcs))]
    check_same(res_g, res_m, dg, dm, "direct encap")
    dgs = datagrams(rng, sessions, 3000, {})
    caps = [max(len(d) - 16, 1) for d in dgs]
    a_in = Arena(dgs, [0] * len(dgs))
    a_out = Arena([b""] * len(dgs), caps)
    for a in (a_in, a_out):
        gpu.register_host(*a.window())
    dm = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
    res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, a_out.ptrs, np.array(caps, np.uint32))
    dg = [bytearray(a_out.get(k, caps[k])) for k in range(len(dgs))]
    check_same(res_g, res_m, dg, dm, "direct decap")
    a_out.buf[:] = 0xEE
    dm = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.decrypt(d, x) for d, x in zip(dgs, dm)]
    res_g = tg.decrypt_ptrs(a_in.ptrs, a_in.lens, a_out.ptrs, np.array(caps, np.uint32))
    dg = [bytearray(a_out.get(k, caps[k])) for k in range(len(dgs))]
    check_same(res_g, res_m, dg, dm, "direct decrypt")
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    for a in (a_src, a_dst, a_in, a_out):
        gpu.unregister_host(a.window()[0])
    tg.close()


@pytest.mark.parametrize("word", ["1", "0"])
def test_small_calls_back_to_back_match_sequential_tunn(gpu, monkeypatch, word):
    """Many back-to-back calls of 1-64 packets (NepTUN's batch size): the latency form
    on the caller's memory, whose completion the host takes from the kernel's own
    completion word (WG_TUNN_FLAG=64: chunks of up to 64 packets) or from the event
    (0).  Staged and registered calls alternate, so consecutive calls share the staging
    sets' words and sequence numbers; every call equals the sequential model."""
    import numpy as np
    monkeypatch.setenv("WG_TUNN_FLAG", "64" if word == "1" else "0")
    rng = random.Random(31 if word == "1" else 32)
    tm, tg, sessions = make_pair(gpu, rng)
    ctr_state = {}
    regs = []
    for call in range(120):
        n = rng.choice([1, 2, 7, 16, 50, 64])
        registered = call % 3 == 2
        if call % 2 == 0:
            srcs = [ipv4(rng, rng.choice([20, 64, 1350, rng.randrange(20, 1500)])) for _ in range(n)]
            caps = [len(s) + 32 for s in srcs]
            dm = [bytearray(b"\xee" * c) for c in caps]
            res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
            if registered:
                a_src, a_dst = Arena(srcs, [0] * n), Arena([b""] * n, caps)
                for a in (a_src, a_dst):
                    gpu.register_host(*a.window())
                    regs.append(a)
                res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, a_dst.ptrs, np.array(caps, np.uint32))
                dg = [bytearray(a_dst.get(k, caps[k])) for k in range(n)]
            else:
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_g = tg.encapsulate_batch(srcs, dg)
            check_same(res_g, res_m, dg, dm, f"encap call {call}")
        else:
            dgs = datagrams(rng, sessions, n, ctr_state)
            caps = [max(len(d) - 16, 1) for d in dgs]
            dm = [bytearray(b"\xee" * c) for c in caps]
            res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
            if registered:
                a_in, a_out = Arena(dgs, [0] * n), Arena([b""] * n, caps)
                for a in (a_in, a_out):
                    gpu.register_host(*a.window())
                    regs.append(a)
                res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, a_out.ptrs, np.array(caps, np.uint32))
                dg = [bytearray(a_out.get(k, caps[k])) for k in range(n)]
            else:
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_g = tg.decapsulate_batch(dgs, dg)
            check_same(res_g, res_m, dg, dm, f"decap call {call}")
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    for a in regs:
        gpu.unregister_host(a.window()[0])
    tg.close()


def test_teardown_and_regrowth_after_word_completed_calls(gpu, torch_cuda, monkeypatch):
    """What can outlive a call in this process, each followed at once by a
    latency-form strided open and a host copy into fresh memory (the shape of the
    round-5 driver fault: test_xlane_gpu's 8192-byte open, then a device-to-host copy):
    a Tunn destroyed right after a word-completed call (no event recorded), staging
    regrown (freed and reallocated) by a large call right after a word-completed one,
    and registered pools unregistered and freed right after a registered small call.
    Every call equals the sequential model; every later launch and copy is clean."""
    import gc

    import numpy as np
    torch = torch_cuda
    monkeypatch.setenv("WG_TUNN_FLAG", "64")
    rng = random.Random(91)

    def xlane_open_then_copy():
        nrng = np.random.default_rng(5)
        key = nrng.integers(0, 256, (1, 32), dtype=np.uint8)
        gpu.set_keys(0, key, np.array([0x1234567], np.uint32))
        n, P, S = 200, 8192, 8224
        src = torch.from_numpy(nrng.integers(0, 256, n * S + 64, dtype=np.uint8)).cuda()
        wire = torch.full((n * S + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        back = torch.full((n * S + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        try:
            gpu.set_xlane_lanes(n * 64)
            gpu.seal_strided(n, P, 0, 7, src, S, wire, S, None)
            gpu.open_strided(n, P + 32, 0, wire, S, back, S, None)
            torch.cuda.synchronize()
        finally:
            gpu.set_xlane_lanes(-1)
        b, s_np = back.cpu().numpy(), src.cpu().numpy()
        w = wire.cpu().numpy()
        for i in (0, n - 1):
            assert w[i * S:i * S + P + 32].tobytes() == o.format_packet_data(
                key[0].tobytes(), 0x1234567, 7 + i, s_np[i * S:i * S + P].tobytes())
        assert np.array_equal(b[:n * S].reshape(n, S)[:, :P], s_np[:n * S].reshape(n, S)[:, :P])

    def small_calls(tm, tg, sessions, ctr_state, n=50):
        srcs = [ipv4(rng, rng.choice([64, 1350])) for _ in range(n)]
        caps = [len(x) + 32 for x in srcs]
        dm, dg = [bytearray(b"\xee" * c) for c in caps], [bytearray(b"\xee" * c) for c in caps]
        check_same(tg.encapsulate_batch(srcs, dg), [tm.encapsulate(x, d) for x, d in zip(srcs, dm)], dg, dm,
                   "small encap")
        dgs = datagrams(rng, sessions, n, ctr_state)
        caps = [max(len(d) - 16, 1) for d in dgs]
        dm, dg = [bytearray(b"\xee" * c) for c in caps], [bytearray(b"\xee" * c) for c in caps]
        check_same(tg.decapsulate_batch(dgs, dg), [tm.decapsulate(d, x) for d, x in zip(dgs, dm)], dg, dm,
                   "small decap")

    # 1. destroyed right after a word-completed call (and collected at once)
    tm, tg, sessions = make_pair(gpu, rng)
    small_calls(tm, tg, sessions, {})
    tg.close()
    del tg
    gc.collect()
    xlane_open_then_copy()
    # 2. staging regrown right after a word-completed call, then small calls again
    tm, tg, sessions = make_pair(gpu, rng)
    st = {}
    small_calls(tm, tg, sessions, st)
    big = [ipv4(rng, 1350) for _ in range(40000)]
    dm, dg = [bytearray(1382) for _ in big], [bytearray(1382) for _ in big]
    check_same(tg.encapsulate_batch(big, dg), [tm.encapsulate(x, d) for x, d in zip(big, dm)], dg, dm, "big")
    small_calls(tm, tg, sessions, st)
    xlane_open_then_copy()
    # 3. registered pools freed right after a registered small call
    srcs = [ipv4(rng, 1350) for _ in range(50)]
    caps = [len(x) + 32 for x in srcs]
    a_src, a_dst = Arena(srcs, [0] * 50), Arena([b""] * 50, caps)
    for a in (a_src, a_dst):
        gpu.register_host(*a.window())
    dm = [bytearray(b"\xee" * c) for c in caps]
    res_m = [tm.encapsulate(x, d) for x, d in zip(srcs, dm)]
    res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, a_dst.ptrs, np.array(caps, np.uint32))
    check_same(res_g, res_m, [bytearray(a_dst.get(k, caps[k])) for k in range(50)], dm, "registered small")
    for a in (a_src, a_dst):
        gpu.unregister_host(a.window()[0])
    del a_src, a_dst, a
    gc.collect()
    xlane_open_then_copy()
    tg.close()


@pytest.mark.parametrize("chunk_kb", [None, "64"])
def test_multi_engine_split_matches_sequential_tunn(torch_cuda, monkeypatch, chunk_kb):
    """wg_tunn_create_multi over two contexts on device 0 (the 1-GPU stand-in for
    one context per GPU): every batch is split into two byte-balanced shares that
    run concurrently on their own driver threads, streams and pinned staging, after
    ONE counter reservation (session.rs:219).  Results, destination bytes,
    counters, replay windows and stats equal N sequential calls of the model.
    With 64 KiB chunks (WG_TUNN_CHUNK_KB) a batch is far larger than one chunk per
    engine: decapsulate then runs in rounds of 2 x 64 KiB, decided in packet order
    across rounds and engines, with no more pinned staging than one chunk."""
    if chunk_kb:
        monkeypatch.setenv("WG_TUNN_CHUNK_KB", chunk_kb)
    from neptun_amd import GpuContext
    from neptun_amd.tunn import Tunn
    rng = random.Random(51)
    ctxs = [GpuContext(0, key_slots=64), GpuContext(0, key_slots=64)]
    tm, tg = M.Tunn(), Tunn(ctxs, 16)
    eng = tg.engines()
    assert len(eng) == 2 and all(d == 0 and n >= -1 for d, n in eng)
    sessions = []
    for j, local in enumerate((5, 22)):
        rk, sk, peer = rng.randbytes(32), rng.randbytes(32), rng.getrandbits(32)
        for t in (tm, tg):
            t.set_time(10 * (j + 1))
            t.install_session(local, peer, rk, sk, True)
        sessions.append((local, peer, rk, sk))
    ctr_state = {}
    for batch in range(3):
        srcs = [ipv4(rng, rng.choice([64, 1350, rng.randrange(20, 1500)])) for _ in range(2500)]
        srcs += [rng.randbytes(rng.choice([0, 17, 8900])) for _ in range(50)]
        rng.shuffle(srcs)
        caps = [len(s) + 32 if rng.random() > 0.02 else len(s) + 20 for s in srcs]
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
        check_same(tg.encapsulate_batch(srcs, dg), res_m, dg, dm, f"multi encap {batch}")
        dgs = datagrams(rng, sessions, 2500, ctr_state)
        caps = [max(len(d) - 16, 0) if rng.random() > 0.02 else max(len(d) - 20, 0) for d in dgs]
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
        check_same(tg.decapsulate_batch(dgs, dg), res_m, dg, dm, f"multi decap {batch}")
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [tm.decrypt(d, x) for d, x in zip(dgs, dm)]
        check_same(tg.decrypt_batch(dgs, dg), res_m, dg, dm, f"multi decrypt {batch}")
    for local, *_ in sessions:
        ctr, w = tg.session_counters(local % M.N_SESSIONS)
        sm = tm.sessions[local % M.N_SESSIONS]
        assert ctr == sm.sending_counter
        assert w.next == sm.window.next and list(w.bitmap) == sm.window.bitmap
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("out", ["scatter", "direct", "auto"])
def test_multi_engine_registered_pools_match_sequential_tunn(torch_cuda, monkeypatch, out):
    """wg_tunn_create_multi over two contexts with the caller's pools registered on both
    (one pin shared by the contexts): each engine runs its share of a batch as a DMA
    batch of its own -- encapsulate after the one counter reservation, decapsulate with
    the replay speculation taken for the whole batch in packet order first and every
    chunk's decisions, repairs and copy-out in packet order once both engines are back --
    in each output form (WG_TUNN_DMA_OUT).  Damage as in the one-engine slot-pool test
    (replays, old counters, forged tags ahead of the real packet, wrong indices,
    keepalives).  Results, dst bytes, windows and stats equal the sequential model's."""
    import numpy as np

    from neptun_amd import GpuContext
    from neptun_amd.tunn import Tunn
    monkeypatch.setenv("WG_TUNN_DMA", "1")
    monkeypatch.setenv("WG_TUNN_DMA_MIN", "0")  # (DMA batches for encapsulate at this size too)
    if out != "auto":
        monkeypatch.setenv("WG_TUNN_DMA_OUT", out)
    monkeypatch.setenv("WG_TUNN_CHUNK_KB", "2048")
    rng = random.Random(57)
    ctxs = [GpuContext(0, key_slots=64), GpuContext(0, key_slots=64)]
    tm, tg = M.Tunn(), Tunn(ctxs, 16)
    sessions = []
    for j, local in enumerate((5, 22)):
        rk, sk, peer = rng.randbytes(32), rng.randbytes(32), rng.getrandbits(32)
        for t in (tm, tg):
            t.set_time(10 * (j + 1))
            t.install_session(local, peer, rk, sk, True)
        sessions.append((local, peer, rk, sk))
    n, slot = 6000, 1536
    srcs = [ipv4(rng, 1350 if rng.random() > 0.02 else rng.choice([64, 1349, 700])) for _ in range(n)]
    a_src, a_dst = SlotArena(srcs, slot), SlotArena([], slot, n)
    arenas = [a_src, a_dst]
    for a in arenas:
        for c in ctxs:
            c.register_host(*a.window())
    caps = np.full(n, slot, np.uint32)
    dm = [bytearray(b"\xee" * slot) for _ in range(n)]
    res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
    tg.phases(reset=True)
    res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, a_dst.ptrs, caps)
    check_same(res_g, res_m, [bytearray(a_dst.get(k, slot)) for k in range(n)], dm, "multi slot encap")
    ph = tg.phases(reset=True)
    # (prep: the DMA batches' setup -- the staged rounds have none)
    assert ph["calls"] == 1 and ph["chunks"] >= 4 and ph["prep_us"] > 0
    local, peer, rk, sk = sessions[1]
    c = 0
    dgs = []
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
    for at in range(100, n - 10, 997):  # a forged copy ahead of the real packet
        forged = bytearray(dgs[at + 7])
        forged[-1] ^= 0x80
        dgs[at] = bytes(forged)
    at_split = n // 2  # one forgery right at the engines' boundary
    forged = bytearray(dgs[at_split + 3])
    forged[-1] ^= 0x80
    dgs[at_split - 2] = bytes(forged)
    a_in, a_out = SlotArena(dgs, slot), SlotArena([], slot, n)
    arenas += [a_in, a_out]
    for a in (a_in, a_out):
        for cx in ctxs:
            cx.register_host(*a.window())
    dm = [bytearray(b"\xee" * slot) for _ in range(n)]
    res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
    res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, a_out.ptrs, caps)
    assert tg.phases(reset=True)["prep_us"] > 0
    check_same(res_g, res_m, [bytearray(a_out.get(k, slot)) for k in range(n)], dm, "multi slot decap")
    kinds = [r[:2] for r in res_m]
    assert (M.ERR, M.INVALID_AEAD_TAG) in kinds and (M.ERR, M.DUPLICATE_COUNTER) in kinds
    ctr, w = tg.session_counters(local % M.N_SESSIONS)
    sm = tm.sessions[local % M.N_SESSIONS]
    assert w.next == sm.window.next and list(w.bitmap) == sm.window.bitmap
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    tg.close()
    for a in arenas:
        for cx in ctxs:
            cx.unregister_host(a.window()[0])
    for cx in ctxs:
        cx.close()


def large_ipv4_udp_packet():
    """create_large_ipv4_udp_packet (noise/mod.rs:846-853): etherparse IPv4 (192.168.1.2 ->
    192.168.1.3, TTL 5) + UDP (5678 -> 23) around 1400 zero bytes = 1428 bytes."""
    total = 20 + 8 + 1400
    ip = bytearray(20)
    ip[0], ip[2:4], ip[8], ip[9] = 0x45, struct.pack(">H", total), 5, 17
    ip[12:16], ip[16:20] = bytes([192, 168, 1, 2]), bytes([192, 168, 1, 3])
    s = sum(struct.unpack(">10H", bytes(ip)))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    ip[10:12] = struct.pack(">H", ~s & 0xFFFF)
    udp = struct.pack(">HHHH", 5678, 23, 8 + 1400, 0)
    return bytes(ip) + udp + bytes(1400)


def test_long_running_streams_byte_accounting(gpu):
    """test_long_running_streams (noise/mod.rs:1116-1140): 4,000,000 encapsulate ->
    decapsulate round trips of one 1428-byte IPv4/UDP packet between two Tunns, after
    which the reference asserts rx >= 1424 * 4M and tx >= 1424 * 4M (the u64 byte
    counters).  Here as 16 batches of 250,000 through the batch ABI: every result Ok
    and every plaintext back, tx == rx == 4M * (1428 + 32) exactly (message_data_len,
    session.rs:357), and the sender's counter at 4M."""
    import numpy as np
    from neptun_amd.tunn import Tunn
    pkt = large_ipv4_udp_packet()
    P, W = len(pkt), len(pkt) + 32
    a, b = Tunn(gpu, FIRST_SLOT), Tunn(gpu, FIRST_SLOT - 16)
    k1, k2 = bytes(range(32)), bytes(range(32, 64))
    a.install_session(21, 34, k2, k1, True)
    b.install_session(34, 21, k1, k2, True)
    n, batches = 250_000, 16
    S = (W + 15) // 16 * 16
    src = np.frombuffer(pkt, np.uint8).copy()           # one buffer, like the reference
    wire = np.zeros(n * S, np.uint8)
    out = np.zeros(n * S, np.uint8)
    slots = np.arange(n, dtype=np.uint64) * S
    src_ptrs = np.full(n, src.ctypes.data, np.uint64)
    src_lens = np.full(n, P, np.uint32)
    wire_ptrs = wire.ctypes.data + slots
    caps = np.full(n, S, np.uint32)
    wire_lens = np.full(n, W, np.uint32)
    out_ptrs = out.ctypes.data + slots
    want = np.frombuffer(pkt, np.uint8)
    for _ in range(batches):
        res = a.encapsulate_ptrs(src_ptrs, src_lens, wire_ptrs, caps)
        assert all(r[0] == M.WRITE_TO_NETWORK and r[2] == W for r in res)
        res = b.decapsulate_ptrs(wire_ptrs, wire_lens, out_ptrs, caps)
        assert all(r[0] == M.WRITE_TO_TUNNEL and r[2] == P for r in res)
        assert (out.reshape(n, S)[:, :P] == want).all()
    total = n * batches
    tx, _ = a.stats()
    _, rx = b.stats()
    assert rx >= 1424 * total and tx >= 1424 * total  # the reference's assertion
    assert tx == rx == total * W
    ctr, _ = a.session_counters(21 % 8)  # a's session: local index 21
    assert ctr == total
    a.close()
    b.close()


class SlotArena(Arena):
    """Packets in fixed-size slots of one buffer (a gateway's packet pool): the
    layout the Tunn moves as DMA runs (one 2D copy per run of equal-length packets)."""

    def __init__(self, blobs, slot, n=None, fill=0xEE):
        import numpy as np
        n = len(blobs) if n is None else n
        self.caps = [slot] * n
        self.buf = np.full(n * slot + 8192, fill, np.uint8)
        base = self.buf.ctypes.data
        self.pad = (-base) % 4096
        self.offs = (self.pad + slot * np.arange(n)).astype(np.uint64)
        for o, b in zip(self.offs, blobs):
            self.buf[int(o):int(o) + len(b)] = np.frombuffer(b, np.uint8)
        self.ptrs = (base + self.offs).astype(np.uint64)
        self.lens = np.array([len(b) for b in blobs] + [0] * (n - len(blobs)), np.uint32)


@pytest.mark.parametrize("dma", ["1", "1-scatter", "1-direct", "1-nested", "1-early", "0"])
def test_registered_slot_pools_match_sequential_tunn(gpu, monkeypatch, dma):
    """Registered packet pools with fixed slots (WG_TUNN_DMA=1: DMA batches -- input runs
    copied to HBM, then the AEAD kernel writes each packet the speculated replay
    decisions land straight into its dst (direct) or into staging with a scatter kernel
    copying it out: "1" the defaults (encapsulate scatter, decapsulate direct),
    "1-scatter" / "1-direct" both operations one way, "1-nested" every stage of a chunk
    on one stream, "1-early" a batch large enough (20,000) for decapsulate to put its
    first chunk on the device before pass 1 has seen the rest; 0: the zero-copy direct
    kernels), several chunks per batch: mostly 1350-byte packets in order, with a
    sprinkle of other lengths (runs break), replays, too-old counters, tampered tags
    (ring's zeros land in dst), wrong indices and keepalives; one batch with a dst
    outside the registered pool (that batch, or with "1-early" the rest of it after the
    first sixteenth, falls back to staging).
    Results, dst bytes, windows and stats equal the sequential model's."""
    import ctypes

    import numpy as np
    monkeypatch.setenv("WG_TUNN_DMA", dma[0])
    monkeypatch.setenv("WG_TUNN_DMA_MIN", "0")  # (DMA batches for encapsulate at this size too)
    if dma in ("1-scatter", "1-direct"):
        monkeypatch.setenv("WG_TUNN_DMA_OUT", dma[2:])
    if dma == "1-nested":
        monkeypatch.setenv("WG_TUNN_DMA_STREAMS", "0")
    monkeypatch.setenv("WG_TUNN_CHUNK_KB", "2048")
    rng = random.Random(55)
    tm, tg, sessions = make_pair(gpu, rng)
    n, slot = (20000 if dma == "1-early" else 6000), 1536
    srcs = [ipv4(rng, 1350 if rng.random() > 0.02 else rng.choice([64, 1349, 700])) for _ in range(n)]
    a_src, a_dst = SlotArena(srcs, slot), SlotArena([], slot, n)
    for a in (a_src, a_dst):
        gpu.register_host(*a.window())
    caps = np.full(n, slot, np.uint32)
    dm = [bytearray(b"\xee" * slot) for _ in range(n)]
    res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
    tg.phases(reset=True)
    res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, a_dst.ptrs, caps)
    check_same(res_g, res_m, [bytearray(a_dst.get(k, slot)) for k in range(n)], dm, "slot encap")
    ph = tg.phases(reset=True)
    assert ph["calls"] == 1 and ph["packets"] == n and ph["chunks"] >= (4 if dma[0] == "1" else 1)
    # inbound: the peer's traffic on session 0, in order with damage sprinkled in
    local, peer, rk, sk = sessions[0]
    state = {"c": 0}

    def inbound():
        dgs = []
        for _ in range(n):
            c = state["c"]
            r = rng.random()
            P = 1350 if rng.random() > 0.02 else rng.choice([0, 64, 1000])
            pt = ipv4(rng, P) if P else b""
            ctr = c if r > 0.03 else max(0, c - rng.randrange(1, 40)) if r > 0.015 else max(0, c - 3000)
            state["c"] = max(c, ctr + 1)
            d = bytearray(o.format_packet_data(rk, local, ctr, pt))
            r = rng.random()
            if r < 0.01:
                d[rng.randrange(16, len(d))] ^= 0x04
            elif r < 0.015:
                d[4:8] = struct.pack("<I", local + 8)
            dgs.append(bytes(d))
        # a forged copy of a counter first, the real packet later: the forgery must not
        # mark the counter, so the real one is accepted (the DMA path's speculation --
        # every tag good -- calls it a duplicate and has to repair it)
        for at in range(100, n - 10, 997):
            ctr = struct.unpack_from("<Q", dgs[at + 7], 8)[0]
            forged = bytearray(dgs[at + 7])
            forged[-1] ^= 0x80
            dgs[at] = bytes(forged)
            assert struct.unpack_from("<Q", dgs[at], 8)[0] == ctr
        return dgs

    for outside in (False, True):
        dgs = inbound()
        a_in, a_out = SlotArena(dgs, slot), SlotArena([], slot, n)
        for a in (a_in, a_out):
            gpu.register_host(*a.window())
        out_ptrs = a_out.ptrs.copy()
        stray = ctypes.create_string_buffer(b"\xee" * slot, slot)
        if outside:  # one accepted packet's dst in ordinary (unregistered) memory
            out_ptrs[4321] = ctypes.addressof(stray)
        dm = [bytearray(b"\xee" * slot) for _ in range(n)]
        res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
        res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, out_ptrs, caps)
        dg = [bytearray(a_out.get(k, slot)) for k in range(n)]
        if outside:
            assert res_m[4321][0] == M.WRITE_TO_TUNNEL or res_m[4321][0] == M.ERR
            dg[4321] = bytearray(stray.raw)
        check_same(res_g, res_m, dg, dm, f"slot decap (a dst outside the pool: {outside})")
        kinds = [r[:2] for r in res_m]
        assert (M.ERR, M.INVALID_AEAD_TAG) in kinds and (M.ERR, M.DUPLICATE_COUNTER) in kinds
        for a in (a_in, a_out):
            gpu.unregister_host(a.window()[0])
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    for a in (a_src, a_dst):
        gpu.unregister_host(a.window()[0])
    tg.close()


@pytest.mark.parametrize("strided", ["1", "0"])
def test_registered_uniform_pools_take_the_strided_open(gpu, monkeypatch, strided):
    """Decapsulate chunks whose packets all land, share one length and sit in line-aligned
    registered slots go through the strided text-grid open straight into dst (the host
    adds the tag bytes); tampered tags keep a chunk on that path (ring's zeros land),
    replays send their chunk to the descriptor kernels.  WG_TUNN_STRIDED=0: every chunk
    on the descriptor kernels.  Results, dst bytes and stats equal the sequential model's."""
    import numpy as np
    monkeypatch.setenv("WG_TUNN_STRIDED", strided)
    monkeypatch.setenv("WG_TUNN_CHUNK_KB", "2048")
    rng = random.Random(77)
    tm, tg, sessions = make_pair(gpu, rng)
    local, peer, rk, sk = sessions[0]
    n, slot = 9000, 1536
    dgs = []
    for c in range(n):
        d = bytearray(o.format_packet_data(rk, local, c, ipv4(rng, 1350)))
        if rng.random() < 0.01:
            d[rng.randrange(16, len(d))] ^= 0x10  # tampered: still lands (zeros)
        dgs.append(bytes(d))
    for at in range(5000, n, 997):  # replays in the second half: those chunks go descriptor
        dgs[at] = dgs[at - 3]
    a_in, a_out = SlotArena(dgs, slot), SlotArena([], slot, n)
    assert int(a_out.ptrs[0]) % 128 == 0
    for a in (a_in, a_out):
        gpu.register_host(*a.window())
    caps = np.full(n, slot, np.uint32)
    dm = [bytearray(b"\xee" * slot) for _ in range(n)]
    res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
    res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, a_out.ptrs, caps)
    check_same(res_g, res_m, [bytearray(a_out.get(k, slot)) for k in range(n)], dm, f"strided {strided}")
    kinds = [r[:2] for r in res_m]
    assert (M.ERR, M.INVALID_AEAD_TAG) in kinds and (M.ERR, M.DUPLICATE_COUNTER) in kinds
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    for a in (a_in, a_out):
        gpu.unregister_host(a.window()[0])
    tg.close()
