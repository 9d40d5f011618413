"""Latency form of the descriptor batches (neptun_amd/csrc/wg_xlane.hip): G lanes
per packet for small batches -- NepTUN's inter-thread batches hold at most 50
packets (/root/reference/neptun/src/device/packet_workers.rs:27).

Each group size G = 64, 32, 16, 8 is forced through wg_gpu_ctx_set_xlane_lanes
(n * G lanes: the largest G that fits is exactly G) and compared bit for bit with
the oracle (oracle/neptun_oracle.c, session.rs:205-302 + RFC 8439) on seal and
open: batch sizes 1, 50, 64 and 1000, payloads 0-9000 bytes including every
block / piece boundary shape, many keys, nonce counters across the 32-bit carry,
and the open failure cases (tampered ciphertext or tag, wrong index, wrong type,
short datagrams, no session) whose plaintext must come back zeroed.
"""
import numpy as np
import pytest

from oracle import pyoracle as o
from tools import synth

from test_gpu_parity import DESC, pack, run_desc

pytestmark = pytest.mark.gpu

EDGE = [0, 1, 15, 16, 17, 47, 48, 63, 64, 65, 111, 112, 127, 128, 129, 191, 192, 1350, 1420,
        4031, 4032, 4033, 8192, 9000]


def make_batch(rng, n, n_keys):
    sizes = rng.integers(0, 9001, n)
    sizes[: min(len(EDGE), n)] = EDGE[: min(len(EDGE), n)]
    rng.shuffle(sizes)
    keys = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, n_keys, dtype=np.uint64).astype(np.uint32)
    payloads = synth.host_payloads(sizes, seed=int(rng.integers(1 << 30)))
    ctrs = rng.integers(0, 2**63, n, dtype=np.uint64) * 2 + rng.integers(0, 2, n, dtype=np.uint64)
    ctrs[: min(4, n)] = [2**32 - 1, 0, 2**32, 2**64 - 1][: min(4, n)]
    slots = rng.integers(0, n_keys, n).astype(np.uint32)
    return sizes, keys, kidx, payloads, ctrs, slots


def seal_descs(sizes, soffs, ctrs, slots, rng):
    n = len(sizes)
    perm = rng.permutation(n)
    doffs = np.zeros(n, np.int64)
    pos = 0
    for i in perm:
        doffs[i] = pos
        pos = synth.round_up(pos + int(sizes[i]) + 32, 16)
    d = np.zeros(n, DESC)
    d["src_off"] = soffs
    d["dst_off"] = doffs
    d["counter"] = ctrs
    d["len"] = sizes
    d["key_slot"] = slots
    return d, pos + 64


@pytest.fixture(scope="module")
def gpu_checked(torch_cuda):
    """A context on the checked build (libneptun_gpu_checked.so: every latency-form
    access checked against its packet's extents, counted and not made)."""
    from neptun_amd import GpuContext, _native
    ctx = GpuContext(0, key_slots=4096, lib_path=_native.CHECKED_LIB_PATH)
    yield ctx
    ctx.close()


@pytest.fixture(params=["product", "checked"])
def xl(request, gpu):
    """Every latency-form test runs on the product library and again on the checked
    build, which must end it with no access outside a packet's own bytes."""
    if request.param == "product":
        yield gpu
        gpu.set_xlane_lanes(-1)  # back to the default selection
        return
    ctx = request.getfixturevalue("gpu_checked")
    ctx.xlane_check(reset=True)
    yield ctx
    ctx.set_xlane_lanes(-1)
    bad = ctx.xlane_check(reset=True)
    assert bad is not None and bad[0] == 0, \
        f"latency form touched memory outside its packet: {bad[0]} accesses, first at {bad[1]:#x} " \
        f"(packet {bad[2]}, lane {bad[3]})"


@pytest.mark.parametrize("G", [64, 32, 16, 8])
@pytest.mark.parametrize("n", [1, 50, 64, 1000])
def test_xlane_seal_open_match_oracle(torch_cuda, xl, G, n):
    torch = torch_cuda
    rng = np.random.default_rng(1000 * G + n)
    sizes, keys, kidx, payloads, ctrs, slots = make_batch(rng, n, 64)
    xl.set_keys(0, keys, kidx)
    xl.set_xlane_lanes(n * G)
    src, soffs = pack(payloads)
    descs, dst_size = seal_descs(sizes, soffs, ctrs, slots, rng)
    out, st = run_desc(torch, xl, True, descs, src, dst_size)
    want = np.zeros(dst_size, np.uint8)
    wst = o.seal_batch(descs, keys, kidx, src, want)
    assert (wst == 0).all()
    assert (st == wst).all(), st
    assert np.array_equal(out, want), "sealed wire bytes differ from the oracle"
    # open the oracle's datagrams back
    d2 = np.zeros(n, DESC)
    d2["src_off"] = descs["dst_off"]
    d2["dst_off"] = soffs
    d2["len"] = sizes + 32
    d2["key_slot"] = slots
    out2, st2 = run_desc(torch, xl, False, d2, want, len(src))
    want2 = np.zeros(len(src), np.uint8)
    wst2 = o.open_batch(d2, keys, kidx, want, want2)
    assert (wst2 == 0).all() and (st2 == 0).all(), st2
    assert np.array_equal(out2, want2)
    assert np.array_equal(out2, src)


@pytest.mark.parametrize("G", [64, 32, 8])
def test_xlane_open_failures_zeroed_like_oracle(torch_cuda, xl, G):
    """Every open failure: status as the oracle's, plaintext of a tag failure
    zeroed, nothing written for the header / slot failures."""
    torch = torch_cuda
    rng = np.random.default_rng(G)
    n = 200
    sizes, keys, kidx, payloads, ctrs, slots = make_batch(rng, n, 16)
    xl.set_keys(0, keys, kidx)
    wires = [o.format_packet_data(keys[slots[i]].tobytes(), int(kidx[slots[i]]), int(ctrs[i]), payloads[i])
             for i in range(n)]
    wires = [bytearray(w) for w in wires]
    slot_col = slots.copy()
    for i in range(n):
        case = i % 10
        w = wires[i]
        if case == 1 and len(w) > 32:
            w[16 + int(rng.integers(len(w) - 32))] ^= 1 << int(rng.integers(8))  # ciphertext
        elif case == 2:
            w[len(w) - 1 - int(rng.integers(16))] ^= 0x80  # tag
        elif case == 3:
            w[4] ^= 1  # receiver index
        elif case == 4:
            w[0] = 1  # handshake type
        elif case == 5:
            wires[i] = w[: int(rng.integers(32))]  # too short for DATA
        elif case == 6:
            slot_col[i] = 0xFFFFFFFF  # no session
        elif case == 7:
            slot_col[i] = 0xFFFFFFFE  # parse failure upstream
    wires = [bytes(w) for w in wires]
    wsrc, woffs = pack(wires)
    out_offs, pos = [], 0
    for w in wires:
        out_offs.append(pos)
        pos = synth.round_up(pos + max(len(w) - 32, 0), 16) + 16
    d = np.zeros(n, DESC)
    d["src_off"] = woffs
    d["dst_off"] = out_offs
    d["len"] = [len(w) for w in wires]
    d["key_slot"] = slot_col
    xl.set_xlane_lanes(n * G)
    d_descs = torch.from_numpy(d.view(np.uint8)).cuda()
    d_src = torch.from_numpy(wsrc).cuda()
    d_dst = torch.full((pos + 64,), 0xAA, dtype=torch.uint8, device="cuda")
    d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    xl.open_batch(d_descs, n, d_src, d_dst, d_st)
    torch.cuda.synchronize()
    st, out = d_st.cpu().numpy(), d_dst.cpu().numpy()
    # the oracle takes the packets that reach a session; the two slot sentinels
    # fail before anything is read (NoCurrentSession / InvalidPacket)
    want = np.full(pos + 64, 0xAA, np.uint8)
    real = slot_col < 0xFFFFFFFE
    wst = np.full(n, -1, np.int32)
    wst[~real] = np.where(slot_col[~real] == 0xFFFFFFFF, 14, 13)
    wst[real] = o.open_batch(d[real], keys, kidx, wsrc, want)
    assert (st == wst).all(), (st, wst)
    assert set(np.unique(wst)) >= {0, 5, 10, 13, 14}
    # the oracle zeroes a tag failure's plaintext and leaves the other failures' bytes
    assert np.array_equal(out, want)
    for i in np.nonzero(wst == 10)[0]:
        p = len(wires[i]) - 32
        assert not out[out_offs[i]:out_offs[i] + p].any()


def test_xlane_in_place_and_absolute_addresses(torch_cuda, xl):
    """In-place open (plaintext over the ciphertext) and null bases (descriptor
    offsets = device addresses), as the throughput forms allow."""
    torch = torch_cuda
    rng = np.random.default_rng(7)
    n = 64
    sizes, keys, kidx, payloads, ctrs, slots = make_batch(rng, n, 4)
    xl.set_keys(0, keys, kidx)
    xl.set_xlane_lanes(n * 64)
    wires = [o.format_packet_data(keys[slots[i]].tobytes(), int(kidx[slots[i]]), int(ctrs[i]), payloads[i])
             for i in range(n)]
    buf, offs = pack(wires)
    d_buf = torch.from_numpy(buf).cuda()
    base = d_buf.data_ptr()
    d = np.zeros(n, DESC)
    d["src_off"] = [base + x for x in offs]
    d["dst_off"] = [base + x + 16 for x in offs]
    d["len"] = [len(w) for w in wires]
    d["key_slot"] = slots
    d_descs = torch.from_numpy(d.view(np.uint8)).cuda()
    d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    xl.open_batch(d_descs, n, None, None, d_st)
    torch.cuda.synchronize()
    assert (d_st.cpu().numpy() == 0).all()
    got = d_buf.cpu().numpy()
    for i in range(n):
        assert got[offs[i] + 16:offs[i] + 16 + len(payloads[i])].tobytes() == payloads[i]


def test_xlane_ordered_launch_matches_unordered(torch_cuda, xl):
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n = 300
    sizes, keys, kidx, payloads, ctrs, slots = make_batch(rng, n, 8)
    xl.set_keys(0, keys, kidx)
    src, soffs = pack(payloads)
    descs, dst_size = seal_descs(sizes, soffs, ctrs, slots, rng)
    want = np.zeros(dst_size, np.uint8)
    o.seal_batch(descs, keys, kidx, src, want)
    xl.set_xlane_lanes(n * 16)
    d_descs = torch.from_numpy(descs.view(np.uint8)).cuda()
    order = torch.from_numpy(rng.permutation(n).astype(np.uint32).view(np.int32)).cuda()
    d_src = torch.from_numpy(src).cuda()
    d_dst = torch.zeros(dst_size, dtype=torch.uint8, device="cuda")
    d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    xl.seal_batch_ordered(d_descs, order, n, d_src, d_dst, d_st)
    torch.cuda.synchronize()
    assert (d_st.cpu().numpy() == 0).all()
    assert np.array_equal(d_dst.cpu().numpy(), want)


@pytest.mark.parametrize("G", [64, 16, 2])
@pytest.mark.parametrize("n,P", [(1, 0), (63, 1350), (64, 17), (200, 8192), (1000, 127)])
def test_xlane_strided_matches_throughput_form_and_oracle(torch_cuda, xl, G, n, P):
    """Strided batches take the latency form too (wg_xlane.hip aead_xlane_strided_kernel):
    every byte of the destination buffer -- packets and the canary bytes around them --
    equals the throughput kernels' output, the sampled datagrams equal the oracle's, and
    the open restores every plaintext (status array optional, as the ABI allows)."""
    torch = torch_cuda
    rng = np.random.default_rng(G * 7 + n + P)
    keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    kidx = np.array([0x1234567], np.uint32)
    xl.set_keys(0, keys, kidx)
    S = synth.round_up(P + 32 + 16 * int(rng.integers(0, 3)), 16)
    src = torch.from_numpy(rng.integers(0, 256, n * S + 64, dtype=np.uint8)).cuda()
    ctr0 = 2**32 - 5
    outs = []
    for lanes in (0, n * G):
        xl.set_xlane_lanes(lanes)
        w = torch.full((n * S + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        xl.seal_strided(n, P, 0, ctr0, src, S, w, S, st)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all()
        outs.append(w)
    assert torch.equal(outs[0], outs[1]), "latency-form seal differs from the throughput form"
    got = outs[1].cpu().numpy()
    s_np = src.cpu().numpy()
    for i in sorted({0, n // 2, n - 1}):
        want = o.format_packet_data(keys[0].tobytes(), int(kidx[0]), ctr0 + i, s_np[i * S:i * S + P].tobytes())
        assert got[i * S:i * S + P + 32].tobytes() == want, i
    back = torch.full((n * S + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    xl.set_xlane_lanes(n * G)
    xl.open_strided(n, P + 32, 0, outs[1], S, back, S, None)
    torch.cuda.synchronize()
    b = back.cpu().numpy()
    for i in range(n):
        assert b[i * S:i * S + P].tobytes() == s_np[i * S:i * S + P].tobytes(), i
        assert (b[i * S + P:(i + 1) * S] == 0x5A).all(), i


@pytest.mark.parametrize("srv", ["0", "1"])
def test_tunn_small_calls_on_the_checked_build(gpu_checked, monkeypatch, srv):
    """The Tunn's small calls -- the latency form with descriptors in the kernel
    arguments (LDS-staged: packets in host memory), the completion word, registered
    datagrams read and registered dsts written in place on speculated replay decisions
    -- and, srv = 1, the same calls posted to the engine's resident kernel, on the
    checked build: every call equals the sequential model and no access leaves its
    packet."""
    import random

    from test_tunn_gpu import Arena, check_same, datagrams, ipv4, make_pair
    monkeypatch.setenv("WG_TUNN_FLAG", "64")
    monkeypatch.setenv("WG_TUNN_SRV", srv)
    ctx = gpu_checked
    ctx.xlane_check(reset=True)
    rng = random.Random(606)
    tm, tg, sessions = make_pair(ctx, rng)
    ctr_state, regs = {}, []
    for call in range(60):
        n = rng.choice([1, 7, 16, 50, 64])
        registered = call % 3 != 0
        if call % 2 == 0:
            srcs = [ipv4(rng, rng.choice([20, 64, 1350, rng.randrange(20, 1500)])) for _ in range(n)]
            caps = [len(s) + 32 for s in srcs]
            dm = [bytearray(b"\xee" * c) for c in caps]
            res_m = [tm.encapsulate(s, d) for s, d in zip(srcs, dm)]
            if registered:
                a_src, a_dst = Arena(srcs, [0] * n), Arena([b""] * n, caps)
                for a in (a_src, a_dst):
                    ctx.register_host(*a.window())
                    regs.append(a)
                res_g = tg.encapsulate_ptrs(a_src.ptrs, a_src.lens, a_dst.ptrs, np.array(caps, np.uint32))
                dg = [bytearray(a_dst.get(k, caps[k])) for k in range(n)]
            else:
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_g = tg.encapsulate_batch(srcs, dg)
            check_same(res_g, res_m, dg, dm, f"checked encap {call}")
        else:
            dgs = datagrams(rng, sessions, n, ctr_state)
            caps = [max(len(d) - 16, 1) for d in dgs]
            dm = [bytearray(b"\xee" * c) for c in caps]
            res_m = [tm.decapsulate(d, x) for d, x in zip(dgs, dm)]
            if registered:
                a_in, a_out = Arena(dgs, [0] * n), Arena([b""] * n, caps)
                for a in (a_in, a_out):
                    ctx.register_host(*a.window())
                    regs.append(a)
                res_g = tg.decapsulate_ptrs(a_in.ptrs, a_in.lens, a_out.ptrs, np.array(caps, np.uint32))
                dg = [bytearray(a_out.get(k, caps[k])) for k in range(n)]
            else:
                dg = [bytearray(b"\xee" * c) for c in caps]
                res_g = tg.decapsulate_batch(dgs, dg)
            check_same(res_g, res_m, dg, dm, f"checked decap {call}")
    assert tg.stats() == (tm.tx_bytes, tm.rx_bytes)
    for a in regs:
        ctx.unregister_host(a.window()[0])
    tg.close()
    bad = ctx.xlane_check(reset=True)
    assert bad[0] == 0, f"{bad[0]} accesses outside their packet, first at {bad[1]:#x} (packet {bad[2]})"
