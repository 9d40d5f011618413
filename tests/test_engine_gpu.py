"""Shared per-GPU engine (wg_engine) and multi-peer batches (wg_tunn_*_multi).

NepTUN keeps one Tunn per peer (/root/reference/neptun/src/device/peer.rs:29) and its
PacketWorkers batch packets of MANY peers into one inter-thread batch
(device/packet_workers.rs:178-233, device/mod.rs:1328-1337).  Here any number of
Tunns attach to one engine without adding threads or streams, and a multi-peer batch
must return exactly what the sequential per-peer calls of oracle/tunn_model.py return:
each Tunn's counters in the order of its packets, its replay window and current
session driven by its packets in order, tx / rx bytes credited to the packet's Tunn.
"""
import os
import random
import struct
import threading

import numpy as np
import pytest

from oracle import tunn_model as M
from oracle import pyoracle as o

from test_tunn_gpu import Arena, check_same, datagrams, ipv4, plaintexts

pytestmark = pytest.mark.gpu


def threads_now():
    return len(os.listdir("/proc/self/task"))


@pytest.fixture(scope="module")
def big_ctx(torch_cuda):
    """4096 Tunns x 16 key slots."""
    from neptun_amd import GpuContext
    ctx = GpuContext(0, key_slots=4096 * 16)
    yield ctx
    ctx.close()


def peers_with_sessions(rng, eng, count, first=0, sessions=(1, 2), none_every=0):
    """count (model, GPU) Tunn pairs on engine eng, each with 1-2 sessions (ring slots
    differ per session); every none_every-th pair gets no session at all."""
    out = []
    for p in range(count):
        tm, tg = M.Tunn(), eng.tunn((first + p) * 16)
        ses = []
        if not (none_every and p % none_every == none_every - 1):
            for j in range(rng.choice(sessions)):
                local = (p * 8 + j * 3 + 1) & 0xFFFFFFFF
                rk, sk, peer = rng.randbytes(32), rng.randbytes(32), rng.getrandbits(32)
                for t in (tm, tg):
                    t.set_time(10 * (j + 1))
                    t.install_session(local, peer, rk, sk, True)
                ses.append((local, peer, rk, sk))
        out.append((tm, tg, ses))
    return out


def check_state(pairs):
    for tm, tg, ses in pairs:
        for local, *_ in ses:
            ctr, w = tg.session_counters(local % M.N_SESSIONS)
            sm = tm.sessions[local % M.N_SESSIONS]
            assert ctr == sm.sending_counter
            assert w.next == sm.window.next and list(w.bitmap) == sm.window.bitmap
            assert w.receive_cnt == sm.window.receive_cnt
        assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)


def test_tunns_on_one_engine_add_no_threads_or_streams(big_ctx):
    """4096 Tunns attach to one engine: no thread and no stream per Tunn; lanes are made
    by batches (one for sequential calls), and wg_tunn_create shares the context's
    default engine."""
    from neptun_amd import Engine, Tunn
    before = threads_now()
    eng = Engine(big_ctx)
    info = eng.info()
    assert info["tunns"] == 0 and info["lanes"] == 0 and info["streams"] == 0
    pool = info["pool_threads"]
    assert 1 <= pool <= 16
    after_engine = threads_now()
    assert after_engine - before == pool - 1  # the pool's workers (the caller is the last part)
    tunns = [eng.tunn(16 * k) for k in range(4096)]
    info = eng.info()
    assert info["tunns"] == 4096 and info["lanes"] == 0 and info["streams"] == 0
    assert threads_now() == after_engine
    rng = random.Random(3)
    for k in (0, 4095):
        tunns[k].install_session(100 + k, 7, rng.randbytes(32), rng.randbytes(32), True)
    for k in (0, 4095, 0):
        srcs = [ipv4(rng, 100) for _ in range(40)]
        res = tunns[k].encapsulate_batch(srcs, [bytearray(200) for _ in srcs])
        assert all(r[0] == M.WRITE_TO_NETWORK for r in res)
    res = eng.encapsulate_multi([tunns[0], tunns[4095]] * 20, [ipv4(rng, 60)] * 40,
                                [bytearray(100) for _ in range(40)])
    assert all(r[0] == M.WRITE_TO_NETWORK for r in res)
    info = eng.info()
    assert info["lanes"] == 1 and info["streams"] == 8 and info["tunns"] == 4096
    assert threads_now() <= after_engine + 4  # (the HIP runtime may start a helper of its own)
    # a Tunn of another engine cannot join this engine's multi-peer batch
    other = Engine(big_ctx)
    from neptun_amd import NeptunGpuError
    # key slots are the context's: a range a live Tunn holds is refused, whatever engine
    with pytest.raises(NeptunGpuError, match="overlap"):
        other.tunn(8)
    tunns[4095].close()  # (its slots are free again)
    stray = other.tunn(16 * 4095)
    with pytest.raises(NeptunGpuError, match="not on this engine"):
        eng.encapsulate_multi([tunns[0], stray], [b"x", b"y"], [bytearray(64), bytearray(64)])
    with pytest.raises(NeptunGpuError, match="still attached"):
        other.close()
    stray.close()
    other.close()
    for t in tunns:
        t.close()
    assert eng.info()["tunns"] == 0
    eng.close()
    # wg_tunn_create: the context's default engine, shared by its Tunns
    a, b = Tunn(big_ctx, 0), Tunn(big_ctx, 16)
    lib = a._lib
    ea, eb = lib.wg_tunn_engine(a._h), lib.wg_tunn_engine(b._h)
    assert ea and ea == eb
    assert a.engines() == [(0, -1)]
    a.close()
    b.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_multi_peer_batches_match_sequential_tunns(big_ctx, seed):
    """64 Tunns, packets of all of them interleaved in every batch (and some Tunns
    without a session): encapsulate_multi / decapsulate_multi == the model's
    per-peer sequential calls in packet order."""
    from neptun_amd import Engine
    rng = random.Random(seed)
    eng = Engine(big_ctx)
    pairs = peers_with_sessions(rng, eng, 64, none_every=16)
    ctr_state = [dict() for _ in pairs]
    for batch in range(3):
        who = [rng.randrange(len(pairs)) for _ in range(3000)]
        srcs = plaintexts(rng, len(who))
        caps = []
        for s in srcs:
            r = rng.random()
            caps.append(len(s) + 32 + rng.randrange(0, 40) if r > 0.05 else
                        len(s) + 16 + rng.randrange(0, 16) if r > 0.02 else len(s) + rng.randrange(0, 16))
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [pairs[p][0].encapsulate(s, d) for p, s, d in zip(who, srcs, dm)]
        res_g = eng.encapsulate_multi([pairs[p][1] for p in who], srcs, dg)
        check_same(res_g, res_m, dg, dm, f"encap multi {batch}")
        # inbound: each packet from its peer's sessions (replays, reorder, tamper, foreign)
        who = [rng.randrange(len(pairs)) for _ in range(3000)]
        dgs = []
        for p in who:
            ses = pairs[p][2]
            dgs += datagrams(rng, ses, 1, ctr_state[p]) if ses else [o.format_packet_data(
                rng.randbytes(32), 5, 0, ipv4(rng, 40))]
        caps = [max(len(d) - 16, 0) if rng.random() > 0.03 else max(len(d) - 20, 0) for d in dgs]
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [pairs[p][0].decapsulate(d, x) for p, d, x in zip(who, dgs, dm)]
        res_g = eng.decapsulate_multi([pairs[p][1] for p in who], dgs, dg)
        check_same(res_g, res_m, dg, dm, f"decap multi {batch}")
        kinds = {r[0] for r in res_m}
        assert {M.WRITE_TO_TUNNEL, M.ERR}.issubset(kinds)
    check_state(pairs)
    # the single-Tunn calls continue where the multi-peer ones left each Tunn
    tm, tg, ses = pairs[0]
    srcs = [ipv4(rng, 300) for _ in range(50)]
    dm = [bytearray(400) for _ in srcs]
    dg = [bytearray(400) for _ in srcs]
    check_same(tg.encapsulate_batch(srcs, dg), [tm.encapsulate(s, d) for s, d in zip(srcs, dm)], dg, dm, "single")
    check_state(pairs)
    for _, tg, _ in pairs:
        tg.close()
    eng.close()


def test_config4_peers_interleaved_round_trip(big_ctx):
    """BASELINE config 4's shape as Tunns: 4096 peers x 64 packets, interleaved, through
    ONE encapsulate_multi and ONE decapsulate_multi (on the peers' mirror Tunns), every
    result and byte against the model; every peer's counters are exactly 0..63."""
    from neptun_amd import Engine
    rng = random.Random(44)
    eng = Engine(big_ctx)
    n_peers, per = 4096, 64
    a_m, a_g, b_m, b_g = [], [], [], []
    for p in range(n_peers):
        k1, k2 = rng.randbytes(32), rng.randbytes(32)
        ia, ib = 1 + 2 * p, 2 + 2 * p
        for t, args in ((M.Tunn(), (ia, ib, k2, k1)), (eng.tunn(16 * p), (ia, ib, k2, k1))):
            t.install_session(*args, True)
            (a_m if isinstance(t, M.Tunn) else a_g).append(t)
    # the receiving side: 4096 more Tunns would need 2 x 4096 x 16 slots -- the model's
    # side B runs on the CPU, the GPU's side B reuses the slots after side A is done
    who = [p for p in range(n_peers) for _ in range(per)]
    rng.shuffle(who)
    srcs = [ipv4(rng, rng.choice([20, 64, 200, rng.randrange(20, 300)])) for _ in who]
    caps = [len(s) + 32 for s in srcs]
    dm = [bytearray(c) for c in caps]
    dg = [bytearray(c) for c in caps]
    res_m = [a_m[p].encapsulate(s, d) for p, s, d in zip(who, srcs, dm)]
    res_g = eng.encapsulate_multi([a_g[p] for p in who], srcs, dg)
    check_same(res_g, res_m, dg, dm, "config 4 encap")
    for p in (0, 1, 4095):
        assert a_g[p].session_counters((1 + 2 * p) % M.N_SESSIONS)[0] == per
    tx = [t.stats()[0] for t in a_g]
    assert tx == [t.tx_bytes for t in a_m]
    for t in a_g:
        t.close()
    for p in range(n_peers):
        k1, k2 = a_m[p].sessions[(1 + 2 * p) % 8].send_key, a_m[p].sessions[(1 + 2 * p) % 8].recv_key
        ia, ib = 1 + 2 * p, 2 + 2 * p
        for t in (M.Tunn(), eng.tunn(16 * p)):
            t.install_session(ib, ia, k1, k2, True)
            (b_m if isinstance(t, M.Tunn) else b_g).append(t)
    wires = [bytes(d[:r[2]]) for d, r in zip(dm, res_m)]
    order = list(range(len(wires)))
    rng.shuffle(order)  # (arrival order differs from send order: reordering inside the window)
    who2 = [who[i] for i in order]
    wires2 = [wires[i] for i in order]
    caps = [len(w) - 16 for w in wires2]
    dm = [bytearray(b"\xee" * c) for c in caps]
    dg = [bytearray(b"\xee" * c) for c in caps]
    res_m = [b_m[p].decapsulate(w, x) for p, w, x in zip(who2, wires2, dm)]
    res_g = eng.decapsulate_multi([b_g[p] for p in who2], wires2, dg)
    check_same(res_g, res_m, dg, dm, "config 4 decap")
    assert all(r[0] == M.WRITE_TO_TUNNEL for r in res_m)
    assert [t.stats()[1] for t in b_g] == [t.rx_bytes for t in b_m]
    for t in b_g:
        t.close()
    eng.close()


def test_registered_multi_peer_batches_match_sequential_tunns(big_ctx, monkeypatch):
    """Registered pools: a multi-peer batch takes the DMA path (copy-engine input runs,
    per-packet key slots and counters in the descriptors, speculated replay decisions
    per Tunn); 20,000 packets over 32 Tunns in 1 MiB chunks, against the model."""
    from neptun_amd import Engine
    monkeypatch.setenv("WG_TUNN_CHUNK_KB", "1024")
    rng = random.Random(61)
    eng = Engine(big_ctx)
    pairs = peers_with_sessions(rng, eng, 32, first=100)
    who = [rng.randrange(32) for _ in range(20000)]
    srcs = [ipv4(rng, rng.choice([64, 1350, rng.randrange(20, 1500)])) for _ in who]
    caps = [len(s) + 32 + rng.randrange(0, 3) * 16 for s in srcs]
    a_src, a_dst = Arena(srcs, [0] * len(srcs)), Arena([b""] * len(srcs), caps)
    for a in (a_src, a_dst):
        big_ctx.register_host(*a.window())
    th = np.array([pairs[p][1]._h.value for p in who], np.uint64)
    dm = [bytearray(b"\xee" * c) for c in caps]
    res_m = [pairs[p][0].encapsulate(s, d) for p, s, d in zip(who, srcs, dm)]
    res_g = eng.encapsulate_multi_ptrs(th, a_src.ptrs, a_src.lens, a_dst.ptrs, np.array(caps, np.uint32))
    check_same(res_g, res_m, [bytearray(a_dst.get(k, caps[k])) for k in range(len(srcs))], dm, "reg encap")
    ctr_state = [dict() for _ in pairs]
    who = [rng.randrange(32) for _ in range(20000)]
    dgs = []
    for p in who:
        dgs += datagrams(rng, pairs[p][2], 1, ctr_state[p])
    caps = [max(len(d) - 16, 1) for d in dgs]
    a_in, a_out = Arena(dgs, [0] * len(dgs)), Arena([b""] * len(dgs), caps)
    for a in (a_in, a_out):
        big_ctx.register_host(*a.window())
    th = np.array([pairs[p][1]._h.value for p in who], np.uint64)
    dm = [bytearray(b"\xee" * c) for c in caps]
    res_m = [pairs[p][0].decapsulate(d, x) for p, d, x in zip(who, dgs, dm)]
    res_g = eng.decapsulate_multi_ptrs(th, a_in.ptrs, a_in.lens, a_out.ptrs, np.array(caps, np.uint32))
    check_same(res_g, res_m, [bytearray(a_out.get(k, caps[k])) for k in range(len(dgs))], dm, "reg decap")
    check_state(pairs)
    for a in (a_src, a_dst, a_in, a_out):
        big_ctx.unregister_host(a.window()[0])
    for _, tg, _ in pairs:
        tg.close()
    eng.close()


def test_concurrent_calls_share_the_engine(big_ctx):
    """8 threads, each with its own Tunn on one engine, call batches at the same time:
    the calls borrow lanes (several in flight), the pool is shared, and every Tunn
    still equals its model."""
    from neptun_amd import Engine
    rng = random.Random(71)
    eng = Engine(big_ctx)
    pairs = peers_with_sessions(rng, eng, 8, first=300, sessions=(2,))
    errors = []
    seeds = [rng.getrandbits(32) for _ in pairs]

    def work(k):
        try:
            r = random.Random(seeds[k])
            tm, tg, ses = pairs[k]
            ctr_state = {}
            for batch in range(6):
                srcs = [ipv4(r, r.choice([64, 1350, r.randrange(20, 1500)])) for _ in range(r.choice([50, 700, 3000]))]
                dm = [bytearray(len(s) + 32) for s in srcs]
                dg = [bytearray(len(s) + 32) for s in srcs]
                res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
                check_same(tg.encapsulate_batch(srcs, dg), res_m, dg, dm, f"thread {k} encap {batch}")
                dgs = datagrams(r, ses, r.choice([50, 700, 3000]), ctr_state)
                caps = [max(len(d) - 16, 0) for d in dgs]
                dm = [bytearray(b"\xee" * c) for c in caps]
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
                check_same(tg.decapsulate_batch(dgs, dg), res_m, dg, dm, f"thread {k} decap {batch}")
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(pairs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[0]
    check_state(pairs)
    info = eng.info()
    assert 1 <= info["lanes"] <= info["max_lanes"]
    for _, tg, _ in pairs:
        tg.close()
    eng.close()


@pytest.mark.parametrize("depth", ["1", "2"])
def test_concurrent_small_calls_combine_into_shared_launches(big_ctx, monkeypatch, depth):
    """NepTUN's shape: 8 threads, each its own peer's Tunn on one engine, calls of 1-64
    packets (staged and registered, encapsulate and decapsulate with damaged traffic)
    at the same time.  Concurrent calls of one direction go out in shared launches
    (the engine's combiner, WG_COMBINE_DEPTH in flight) -- and every call still equals
    its peer's sequential model."""
    from neptun_amd import Engine

    from test_tunn_gpu import Arena
    monkeypatch.setenv("WG_TUNN_FLAG", "64")
    monkeypatch.setenv("WG_TUNN_SRV", "0")  # (the resident service would take these calls)
    monkeypatch.setenv("WG_COMBINE", "1")  # (off by default: DESIGN 8)
    monkeypatch.setenv("WG_COMBINE_DEPTH", depth)
    rng = random.Random(808 + int(depth))
    eng = Engine(big_ctx)
    pairs = peers_with_sessions(rng, eng, 8, first=600, sessions=(1, 2))
    errors = []
    seeds = [rng.getrandbits(32) for _ in pairs]

    def work(k):
        try:
            r = random.Random(seeds[k])
            tm, tg, ses = pairs[k]
            ctr_state = {}
            for call in range(150):
                n = r.choice([1, 16, 50, 50, 64])
                reg = call % 3 == 1
                if call % 2 == 0:
                    srcs = [ipv4(r, r.choice([64, 1350, r.randrange(20, 1500)])) for _ in range(n)]
                    caps = [len(x) + 32 for x in srcs]
                    dm = [bytearray(b"\xee" * c) for c in caps]
                    res_m = [tm.encapsulate(x, d) for x, d in zip(srcs, dm)]
                    if reg:
                        a, b = Arena(srcs, [0] * n), Arena([b""] * n, caps)
                        for x in (a, b):
                            big_ctx.register_host(*x.window())
                        res_g = tg.encapsulate_ptrs(a.ptrs, a.lens, b.ptrs, np.array(caps, np.uint32))
                        dg = [bytearray(b.get(j, caps[j])) for j in range(n)]
                        for x in (a, b):
                            big_ctx.unregister_host(x.window()[0])
                    else:
                        dg = [bytearray(b"\xee" * c) for c in caps]
                        res_g = tg.encapsulate_batch(srcs, dg)
                    check_same(res_g, res_m, dg, dm, f"thread {k} encap {call}")
                else:
                    dgs = datagrams(r, ses, n, ctr_state)
                    caps = [max(len(d) - 16, 1) for d in dgs]
                    dm = [bytearray(b"\xee" * c) for c in caps]
                    res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
                    if reg:
                        a, b = Arena(dgs, [0] * n), Arena([b""] * n, caps)
                        for x in (a, b):
                            big_ctx.register_host(*x.window())
                        res_g = tg.decapsulate_ptrs(a.ptrs, a.lens, b.ptrs, np.array(caps, np.uint32))
                        dg = [bytearray(b.get(j, caps[j])) for j in range(n)]
                        for x in (a, b):
                            big_ctx.unregister_host(x.window()[0])
                    else:
                        dg = [bytearray(b"\xee" * c) for c in caps]
                        res_g = tg.decapsulate_batch(dgs, dg)
                    check_same(res_g, res_m, dg, dm, f"thread {k} decap {call}")
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(pairs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[0]
    check_state(pairs)
    if depth == "1":  # (one launch in flight: calls arriving meanwhile must share the next;
        # with two, whether any call waits for a slot depends on the kernels' speed)
        # The calls above spend most of their time in Python between launches, so whether
        # two overlap is chance; a burst released at one barrier makes 8 calls arrive
        # within microseconds of each other.
        bar = threading.Barrier(len(pairs))

        def burst(k):
            try:
                r = random.Random(seeds[k] ^ 0x5A5A)
                tm, tg, _ = pairs[k]
                for rep in range(20):
                    srcs = [ipv4(r, 1350) for _ in range(50)]
                    caps = [len(x) + 32 for x in srcs]
                    dm = [bytearray(b"\xee" * c) for c in caps]
                    res_m = [tm.encapsulate(x, d) for x, d in zip(srcs, dm)]
                    dg = [bytearray(b"\xee" * c) for c in caps]
                    bar.wait(timeout=60)
                    res_g = tg.encapsulate_batch(srcs, dg)
                    check_same(res_g, res_m, dg, dm, f"thread {k} burst {rep}")
            except Exception as e:  # noqa: BLE001 (reported below)
                errors.append(e)
                bar.abort()

        th = [threading.Thread(target=burst, args=(k,)) for k in range(len(pairs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors[0]
        check_state(pairs)
        assert eng.info()["combined"] > 0, "no two concurrent small calls shared a launch"
    for _, tg, _ in pairs:
        tg.close()
    eng.close()


def _small_call_traffic(big_ctx, pairs, k, seed, calls, rekey_at=None, pause_at=None):
    """calls of 1-64 packets on pair k (staged and registered, encapsulate and decapsulate
    with damaged traffic), each checked against the pair's sequential model; at call
    rekey_at the pair installs a new session (new keys in the context's table), at call
    pause_at the thread sleeps past the service's lease"""
    import time

    from test_tunn_gpu import Arena
    r = random.Random(seed)
    tm, tg, ses = pairs[k]
    ctr_state = {}
    for call in range(calls):
        if call == rekey_at:
            local = (ses[0][0] + 4) & 0xFFFFFFFF
            rk, sk, peer = r.randbytes(32), r.randbytes(32), r.getrandbits(32)
            for t in (tm, tg):
                t.set_time(100 + call)
                t.install_session(local, peer, rk, sk, True)
            ses[:] = [(local, peer, rk, sk)]
            ctr_state.clear()
        if call == pause_at:
            time.sleep(0.06)
        n = r.choice([1, 16, 50, 50, 64])
        reg = call % 3 == 1
        if call % 2 == 0:
            srcs = [ipv4(r, r.choice([64, 1350, r.randrange(20, 1500)])) for _ in range(n)]
            caps = [len(x) + 32 for x in srcs]
            dm = [bytearray(b"\xee" * c) for c in caps]
            res_m = [tm.encapsulate(x, d) for x, d in zip(srcs, dm)]
            if reg:
                a, b = Arena(srcs, [0] * n), Arena([b""] * n, caps)
                for x in (a, b):
                    big_ctx.register_host(*x.window())
                res_g = tg.encapsulate_ptrs(a.ptrs, a.lens, b.ptrs, np.array(caps, np.uint32))
                dg = [bytearray(b.get(j, caps[j])) for j in range(n)]
                for x in (a, b):
                    big_ctx.unregister_host(x.window()[0])
            else:
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_g = tg.encapsulate_batch(srcs, dg)
            check_same(res_g, res_m, dg, dm, f"pair {k} encap {call}")
        else:
            dgs = datagrams(r, ses, n, ctr_state)
            caps = [max(len(d) - 16, 1) for d in dgs]
            dm = [bytearray(b"\xee" * c) for c in caps]
            res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
            if reg:
                a, b = Arena(dgs, [0] * n), Arena([b""] * n, caps)
                for x in (a, b):
                    big_ctx.register_host(*x.window())
                res_g = tg.decapsulate_ptrs(a.ptrs, a.lens, b.ptrs, np.array(caps, np.uint32))
                dg = [bytearray(b.get(j, caps[j])) for j in range(n)]
                for x in (a, b):
                    big_ctx.unregister_host(x.window()[0])
            else:
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_g = tg.decapsulate_batch(dgs, dg)
            check_same(res_g, res_m, dg, dm, f"pair {k} decap {call}")


def test_resident_service_serves_concurrent_small_calls(big_ctx, monkeypatch):
    """The engine's resident kernel (wg_xlane.hip xlane_service_kernel) takes the small
    calls of 8 concurrent threads, each on its own peer's Tunn: every call equals its
    model, across lease renewals (a 20 ms lease here), a key-table update in the middle
    (one peer installs a new session: the kernel is relaunched before the next post,
    so no call reads old keys), and a pause past the lease (the next call relaunches)."""
    from neptun_amd import Engine
    monkeypatch.setenv("WG_TUNN_SRV", "1")  # (off by default)
    monkeypatch.setenv("WG_TUNN_SRV_LEASE_US", "20000")
    rng = random.Random(909)
    eng = Engine(big_ctx)
    pairs = peers_with_sessions(rng, eng, 8, first=700, sessions=(1,))
    errors = []
    seeds = [rng.getrandbits(32) for _ in pairs]

    def work(k):
        try:
            _small_call_traffic(big_ctx, pairs, k, seeds[k], 120, rekey_at=60 if k == 3 else None,
                                pause_at=90 if k == 5 else None)
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    th = [threading.Thread(target=work, args=(k,)) for k in range(len(pairs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[0]
    check_state(pairs)
    info = eng.info()
    # (every call with packets for the GPU is one chunk; a batch whose every datagram
    # fails its header checks sends none)
    assert info["served"] >= 0.9 * 8 * 120, info
    assert info["service_launches"] >= 2, info
    for _, tg, _ in pairs:
        tg.close()
    eng.close()


def test_resident_service_off_matches_too(big_ctx, monkeypatch):
    """WG_TUNN_SRV=0 (the default): the same traffic through one launch per call (the
    staged latency form); nothing served."""
    from neptun_amd import Engine
    monkeypatch.setenv("WG_TUNN_SRV", "0")
    rng = random.Random(910)
    eng = Engine(big_ctx)
    pairs = peers_with_sessions(rng, eng, 1, first=720, sessions=(1,))
    _small_call_traffic(big_ctx, pairs, 0, 77, 60, rekey_at=30)
    check_state(pairs)
    assert eng.info()["served"] == 0
    pairs[0][1].close()
    eng.close()


@pytest.fixture(scope="module")
def two_ctx(torch_cuda):
    """Two contexts on device 0: the 1-GPU stand-in for one engine per GPU."""
    from neptun_amd import GpuContext
    ctxs = [GpuContext(0, key_slots=2049 * 16), GpuContext(0, key_slots=2049 * 16)]
    yield ctxs
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("n_peers", [64, 4096])
def test_multi_peer_batches_across_engines_match_sequential_tunns(two_ctx, n_peers):
    """wg_tunn_*_multi with no engine: the peers' Tunns alternate between two engines
    (two contexts -- on a node, one per GPU), every batch interleaves packets of all of
    them; the call splits it by engine, runs the shares concurrently and returns the
    results in packet order -- equal to the model's per-peer sequential calls, bytes,
    counters, windows and stats (NepTUN's PacketWorkers over every peer,
    packet_workers.rs:113-131, 178-233; one Mutex<Tunn> per peer, device/peer.rs:29)."""
    from neptun_amd import Engine
    from neptun_amd import tunn as T
    rng = random.Random(7000 + n_peers)
    engs = [Engine(c) for c in two_ctx]
    pairs = []
    for p in range(n_peers):
        tm, tg = M.Tunn(), engs[p % 2].tunn((p // 2) * 16)
        ses = []
        if n_peers == 64 and p % 16 == 15:
            pass  # (a peer without a session)
        else:
            for j in range(1 if n_peers > 64 else rng.choice((1, 2))):
                local = (p * 8 + j * 3 + 1) & 0xFFFFFFFF
                rk, sk, peer = rng.randbytes(32), rng.randbytes(32), rng.getrandbits(32)
                for t in (tm, tg):
                    t.set_time(10 * (j + 1))
                    t.install_session(local, peer, rk, sk, True)
                ses.append((local, peer, rk, sk))
        pairs.append((tm, tg, ses))
    ctr_state = [dict() for _ in pairs]
    per = 3000 if n_peers == 64 else 4 * n_peers
    for batch in range(2):
        who = [rng.randrange(n_peers) for _ in range(per)]
        srcs = [ipv4(rng, rng.choice([20, 64, 576, 1350, rng.randrange(20, 1500)])) for _ in who]
        caps = [len(s) + 32 + rng.randrange(0, 3) * 16 for s in srcs]
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [pairs[p][0].encapsulate(s, d) for p, s, d in zip(who, srcs, dm)]
        res_g = T.encapsulate_multi([pairs[p][1] for p in who], srcs, dg)
        check_same(res_g, res_m, dg, dm, f"across encap {batch}")
        who = [rng.randrange(n_peers) for _ in range(per)]
        dgs = []
        for p in who:
            ses = pairs[p][2]
            dgs += datagrams(rng, ses, 1, ctr_state[p]) if ses else [o.format_packet_data(
                rng.randbytes(32), 5, 0, ipv4(rng, 40))]
        caps = [max(len(d) - 16, 0) for d in dgs]
        dm = [bytearray(b"\xee" * c) for c in caps]
        dg = [bytearray(b"\xee" * c) for c in caps]
        res_m = [pairs[p][0].decapsulate(d, x) for p, d, x in zip(who, dgs, dm)]
        res_g = T.decapsulate_multi([pairs[p][1] for p in who], dgs, dg)
        check_same(res_g, res_m, dg, dm, f"across decap {batch}")
    check_state(pairs)
    # concurrent callers on disjoint peer sets: the engines' drivers are contended (a
    # share whose driver another call holds runs on its caller)
    if n_peers == 64:
        errors = []

        def worker(k):
            try:
                r = random.Random(k)
                mine = [p for p in range(n_peers) if p % 4 == k]
                for _ in range(10):
                    who = [r.choice(mine) for _ in range(200)]
                    srcs = [ipv4(r, r.choice([64, 1350])) for _ in who]
                    dm = [bytearray(len(s) + 32) for s in srcs]
                    dg = [bytearray(len(s) + 32) for s in srcs]
                    res_m = [pairs[p][0].encapsulate(s, d) for p, s, d in zip(who, srcs, dm)]
                    res_g = T.encapsulate_multi([pairs[p][1] for p in who], srcs, dg)
                    check_same(res_g, res_m, dg, dm, f"concurrent {k}")
            except Exception as e:  # (reported by the main thread)
                errors.append(e)

        ths = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert not errors, errors[0]
        check_state(pairs)
    # a Tunn of wg_tunn_create_multi (private engines) cannot join an engine-free batch
    from neptun_amd import NeptunGpuError, Tunn
    priv = Tunn(list(two_ctx), 2048 * 16)  # (past the peers' slots)
    with pytest.raises(NeptunGpuError, match="private engines"):
        T.encapsulate_multi([pairs[0][1], priv], [b"x", b"y"], [bytearray(64), bytearray(64)])
    priv.close()
    for _, tg, _ in pairs:
        tg.close()
    for e in engs:
        e.close()


def test_closing_the_context_closes_its_tunns_and_engines_first(torch_cuda):
    """A Tunn, an engine and a pipe still open when their context closes: the context
    closes them first (their native objects refer to it), so nothing is left to touch a
    freed context at garbage collection or interpreter exit."""
    from neptun_amd import Engine, Tunn
    from neptun_amd.gpu import GpuContext, GpuPipe

    ctx = GpuContext(0, key_slots=64)
    eng = Engine(ctx)
    tunns = [Tunn(ctx, first_slot=16 * k, engine=eng) for k in range(2)]
    pipe = GpuPipe(ctx, chunk_bytes=1 << 20, depth=2)
    tunns[0].install_session(7, 9, bytes(32), bytes(range(32)), True)
    ctx.close()
    assert all(t._h is None for t in tunns) and eng._h is None and pipe._h is None
    ctx.close()  # (twice: nothing left to do)
