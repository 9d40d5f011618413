"""Parity of the gfx950 kernels (through the C ABI) with the CPU oracle.

Bit-exact: every wire byte of seal (header | ciphertext | tag,
session.rs:205-259) and every plaintext byte + status of open
(session.rs:265-302) must equal the oracle's on the same keys, counters and
payloads.  Golden fixtures pin both to the reference KAT (handshake.rs:957-992)
and to three independent RFC 8439 implementations (oracle/gen_golden.py).
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as o
from tools import synth

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
DESC = o.DESC_DTYPE


@pytest.fixture(autouse=True)
def throughput_forms(gpu):
    """The descriptor tests here cover the throughput kernels' wave shapes: the latency
    form (G lanes per packet for small batches) is off for them and has its own tests
    (test_xlane_gpu.py); the Tunn and engine tests run with the default selection."""
    gpu.set_xlane_lanes(0)
    yield
    gpu.set_xlane_lanes(-1)


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def to_dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run_desc(torch, gpu, seal, descs, src, dst_size, slot_base=0):
    """Launch a descriptor batch; returns (dst bytes, status) on the host."""
    d_descs = to_dev(torch, descs.view(np.uint8))
    d_src = to_dev(torch, src)
    d_dst = torch.zeros(max(dst_size, 16), dtype=torch.uint8, device="cuda")
    d_st = torch.full((len(descs),), -1, dtype=torch.int32, device="cuda")
    fn = gpu.seal_batch if seal else gpu.open_batch
    fn(d_descs, len(descs), d_src, d_dst, d_st)
    torch.cuda.synchronize()
    return d_dst.cpu().numpy(), d_st.cpu().numpy()


def pack(items, align=16, pad=32):
    """Lay out byte strings at 16-aligned offsets; returns (buffer, offsets)."""
    offs, pos = [], 0
    for b in items:
        offs.append(pos)
        pos = synth.round_up(pos + len(b) + pad, align)
    buf = np.zeros(pos + 64, np.uint8)
    for off, b in zip(offs, items):
        buf[off:off + len(b)] = np.frombuffer(b, np.uint8)
    return buf, offs


def test_golden_vectors_seal_and_open(torch_cuda, gpu):
    torch = torch_cuda
    vecs = golden("data_packets.json")["vectors"]
    n = len(vecs)
    keys = np.stack([np.frombuffer(bytes.fromhex(v["key"]), np.uint8) for v in vecs])
    idx = np.array([v["sending_index"] for v in vecs], np.uint32)
    gpu.set_keys(0, keys, idx)
    payloads = [bytes.fromhex(v["payload"]) for v in vecs]
    src, soffs = pack(payloads)
    wires = [bytes.fromhex(v["wire"]) for v in vecs]
    _, doffs = pack(wires)
    descs = np.zeros(n, DESC)
    for i, v in enumerate(vecs):
        descs[i] = (soffs[i], doffs[i], v["counter"], len(payloads[i]), i)
    dst_size = doffs[-1] + len(wires[-1]) + 64
    out, st = run_desc(torch, gpu, True, descs, src, dst_size)
    assert (st == 0).all()
    for i in range(n):
        got = out[doffs[i]:doffs[i] + len(wires[i])].tobytes()
        assert got == wires[i], f"vector {i} (len {len(payloads[i])}) differs"
    # the bytes between packets were not touched
    mask = np.ones(len(out), bool)
    for i in range(n):
        mask[doffs[i]:doffs[i] + len(wires[i])] = False
    assert not out[mask].any()
    # open what the fixtures hold
    wsrc, woffs = pack(wires)
    descs2 = np.zeros(n, DESC)
    for i in range(n):
        descs2[i] = (woffs[i], soffs[i], 0, len(wires[i]), i)
    out2, st2 = run_desc(torch, gpu, False, descs2, wsrc, len(src))
    assert (st2 == 0).all()
    for i in range(n):
        assert out2[soffs[i]:soffs[i] + len(payloads[i])].tobytes() == payloads[i]


def test_tampered_datagrams_rejected_and_zeroed(torch_cuda, gpu):
    torch = torch_cuda
    vecs = golden("tamper.json")["vectors"]
    n = len(vecs)
    keys = np.stack([np.frombuffer(bytes.fromhex(v["key"]), np.uint8) for v in vecs])
    idx = np.array([v["receiving_index"] for v in vecs], np.uint32)
    gpu.set_keys(0, keys, idx)
    wires = [bytes.fromhex(v["wire"]) for v in vecs]
    wsrc, woffs = pack(wires)
    out_offs, pos = [], 0
    for w in wires:
        out_offs.append(pos)
        pos = synth.round_up(pos + len(w), 16)
    descs = np.zeros(n, DESC)
    for i in range(n):
        descs[i] = (woffs[i], out_offs[i], 0, len(wires[i]), i)
    # pre-fill the destination with 0xAA so "zeroed" is observable
    d_descs = to_dev(torch, descs.view(np.uint8))
    d_src = to_dev(torch, wsrc)
    d_dst = torch.full((pos + 64,), 0xAA, dtype=torch.uint8, device="cuda")
    d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.open_batch(d_descs, n, d_src, d_dst, d_st)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    assert (st == 10).all(), st
    for i in range(n):
        p = len(wires[i]) - 32
        assert not out[out_offs[i]:out_offs[i] + p].any(), vecs[i]["case"]


def random_batch(rng, n, max_len, n_keys):
    sizes = rng.integers(0, max_len + 1, n)
    sizes[:8] = [0, 1, 15, 16, 17, 63, 64, 65][: min(8, n)]
    keys = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, n_keys, dtype=np.uint64).astype(np.uint32)
    payloads = synth.host_payloads(sizes, seed=int(rng.integers(1 << 30)))
    ctrs = rng.integers(0, 2**63, n, dtype=np.uint64) * 2 + rng.integers(0, 2, n, dtype=np.uint64)
    ctrs[:4] = [0, 2**32 - 1, 2**32, 2**64 - 1][: min(4, n)]
    slots = rng.integers(0, n_keys, n).astype(np.uint32)
    return sizes, keys, kidx, payloads, ctrs, slots


@pytest.mark.parametrize("seed,n,max_len,n_keys", [(1, 3000, 9000, 64), (2, 20000, 1500, 4096)])
def test_random_batches_match_oracle(torch_cuda, gpu, seed, n, max_len, n_keys):
    torch = torch_cuda
    rng = np.random.default_rng(seed)
    sizes, keys, kidx, payloads, ctrs, slots = random_batch(rng, n, max_len, n_keys)
    gpu.set_keys(0, keys, kidx)
    src, soffs = pack(payloads)
    # wire slots: shuffled order so neighbouring lanes hit unrelated memory
    perm = rng.permutation(n)
    doffs = np.zeros(n, np.int64)
    pos = 0
    for i in perm:
        doffs[i] = pos
        pos = synth.round_up(pos + int(sizes[i]) + 32, 16)
    dst_size = pos + 64
    descs = np.zeros(n, DESC)
    descs["src_off"] = soffs
    descs["dst_off"] = doffs
    descs["counter"] = ctrs
    descs["len"] = sizes
    descs["key_slot"] = slots
    out, st = run_desc(torch, gpu, True, descs, src, dst_size)
    want = np.zeros(dst_size, np.uint8)
    wst = o.seal_batch(descs, keys, kidx, src, want)
    assert (st == wst).all() and (st == 0).all()
    assert np.array_equal(out, want), "sealed wire bytes differ from the oracle"
    # open the GPU's own output back
    descs2 = np.zeros(n, DESC)
    descs2["src_off"] = doffs
    descs2["dst_off"] = soffs
    descs2["len"] = sizes + 32
    descs2["key_slot"] = slots
    out2, st2 = run_desc(torch, gpu, False, descs2, out, len(src))
    assert (st2 == 0).all()
    assert np.array_equal(out2, src)


def test_strided_matches_oracle_and_counter_carry(torch_cuda, gpu):
    torch = torch_cuda
    n, P, S = 4096, 1350, 1408
    keys = synth.keys(1)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    pt = synth.device_payloads(n, P, S, "cuda")
    wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    back = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    base = 2**32 - 1000  # counters cross 2^32 inside the batch
    gpu.seal_strided(n, P, 0, base, pt, S, wire, S, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    src = pt.cpu().numpy()
    out = wire.cpu().numpy()
    descs = np.zeros(n, DESC)
    descs["src_off"] = np.arange(n) * S
    descs["dst_off"] = np.arange(n) * S
    descs["counter"] = base + np.arange(n, dtype=np.uint64)
    descs["len"] = P
    want = np.zeros_like(out)
    assert (o.seal_batch(descs, keys, np.array([synth.RECEIVER_IDX], np.uint32), src, want) == 0).all()
    rows_out = out.reshape(n, S)[:, :P + 32]
    rows_want = want.reshape(n, S)[:, :P + 32]
    assert np.array_equal(rows_out, rows_want)
    assert not out.reshape(n, S)[:, P + 32:].any()  # nothing written past the packet
    st.fill_(-1)
    gpu.open_strided(n, P + 32, 0, wire, S, back, S, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    assert torch.equal(back.view(n, S)[:, :P], pt.view(n, S)[:, :P])


@pytest.mark.parametrize("P", [1344, 1350, 64])
def test_strided_tightly_packed_slots(torch_cuda, gpu, P):
    """Strides equal to the packet extents (plaintexts back to back at stride P,
    datagrams at stride P + 32, both 16-aligned): the last lane of every wave
    reads and writes right up to the wave's end -- the buffer resource's range
    must cover it exactly (wg_aead.hip stage_in / stage_out num_records)."""
    torch = torch_cuda
    n = 64 * 37 + 5
    Sp, Sw = synth.round_up(P, 16), synth.round_up(P + 32, 16)
    keys = synth.keys(1)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    rng = np.random.default_rng(P)
    src = rng.integers(0, 256, n * Sp + 64, dtype=np.uint8)
    pt = to_dev(torch, src)
    wire = torch.zeros(n * Sw + 64, dtype=torch.uint8, device="cuda")
    back = torch.zeros(n * Sp + 64, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.seal_strided(n, P, 0, 9, pt, Sp, wire, Sw, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    descs = np.zeros(n, DESC)
    descs["src_off"] = np.arange(n) * Sp
    descs["dst_off"] = np.arange(n) * Sw
    descs["counter"] = 9 + np.arange(n, dtype=np.uint64)
    descs["len"] = P
    want = np.zeros(n * Sw + 64, np.uint8)
    assert (o.seal_batch(descs, keys, np.array([synth.RECEIVER_IDX], np.uint32), src, want) == 0).all()
    assert np.array_equal(wire.cpu().numpy(), want)
    st.fill_(-1)
    gpu.open_strided(n, P + 32, 0, wire, Sw, back, Sp, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    got = back.cpu().numpy()
    assert np.array_equal(got[:n * Sp].reshape(n, Sp)[:, :P], src[:n * Sp].reshape(n, Sp)[:, :P])


def test_open_header_checks(torch_cuda, gpu):
    torch = torch_cuda
    v = golden("data_packets.json")["vectors"][23]  # 1350 bytes
    key = np.frombuffer(bytes.fromhex(v["key"]), np.uint8)[None]
    gpu.set_keys(0, key, np.array([v["sending_index"]], np.uint32))
    gpu.set_keys(1, key, np.array([v["sending_index"] ^ 0x100], np.uint32))
    wire = bytearray(bytes.fromhex(v["wire"]))
    bad_type = bytearray(wire)
    bad_type[0] = 2
    items = [bytes(wire), bytes(bad_type), bytes(wire), bytes(wire), bytes(wire), bytes(wire)]
    src, offs = pack(items)
    descs = np.zeros(len(items), DESC)
    for i in range(len(items)):
        descs[i] = (offs[i], 2048 * i, 0, len(items[i]), 0)
    descs[2]["key_slot"] = 1          # receiver index mismatch -> WrongIndex
    descs[3]["len"] = 31              # shorter than a DATA message -> InvalidPacket
    descs[4]["src_off"] += 4          # misaligned
    descs[5]["key_slot"] = 4096       # outside the key table
    _, st = run_desc(torch, gpu, False, descs, src, 2048 * len(items))
    assert list(st) == [0, 13, 5, 13, 100, 101]


def test_in_place_seal_and_open(torch_cuda, gpu):
    """encapsulate_in_place layout: plaintext at slot+16, wire at slot (noise/mod.rs:303-338)."""
    torch = torch_cuda
    n, P, S = 512, 1000, 1056
    keys = synth.keys(1, seed=99)
    gpu.set_keys(0, keys, np.array([7], np.uint32))
    pt = synth.device_payloads(n, P, S - 16, "cuda", seed=5).view(n, S - 16)
    buf = torch.zeros((n, S), dtype=torch.uint8, device="cuda")
    buf[:, 16:] = pt
    ref = buf.clone()
    base = buf.data_ptr()
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.seal_strided(n, P, 0, 77, base + 16, S, base, S, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    src = ref.cpu().numpy().reshape(-1)
    want = np.zeros_like(src)
    descs = np.zeros(n, DESC)
    descs["src_off"] = np.arange(n) * S + 16
    descs["dst_off"] = np.arange(n) * S
    descs["counter"] = 77 + np.arange(n, dtype=np.uint64)
    descs["len"] = P
    o.seal_batch(descs, keys, np.array([7], np.uint32), src, want)
    got = buf.cpu().numpy()
    assert np.array_equal(got[:, :P + 32], want.reshape(n, S)[:, :P + 32])
    # open in place: plaintext lands at slot+16 (over the ciphertext)
    gpu.open_strided(n, P + 32, 0, base, S, base + 16, S, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    assert torch.equal(buf[:, 16:16 + P], ref[:, 16:16 + P])


def test_config2_full_size_round_trip(torch_cuda, gpu):
    """1M x 1350 B (BASELINE config 2): seal->open identity, status, and EVERY sealed
    datagram equal to the oracle's (chunked host comparison, tests/oracle_chunks.py);
    then one 64 Ki-packet chunk of oracle-sealed datagrams (other payloads, other
    counters) spliced into the batch is opened by the GPU back to the oracle's
    plaintext -- the open kernel checked on bytes it did not produce itself."""
    torch = torch_cuda
    from oracle_chunks import seal_matches_oracle
    n, P, S = 1 << 20, 1350, 1408
    keys = synth.keys(1)
    kidx = np.array([synth.RECEIVER_IDX], np.uint32)
    gpu.set_keys(0, keys, kidx)
    pt = synth.device_payloads(n, P, S, "cuda")
    wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    back = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.seal_strided(n, P, 0, 0, pt, S, wire, S, st)
    gpu.open_strided(n, P + 32, 0, wire, S, back, S, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert torch.equal(back.view(n, S)[:, :P], pt.view(n, S)[:, :P])
    descs = np.zeros(n, DESC)
    descs["src_off"] = descs["dst_off"] = np.arange(n, dtype=np.int64) * S
    descs["counter"] = np.arange(n, dtype=np.uint64)
    descs["len"] = P
    r = seal_matches_oracle(pt, wire, descs, np.arange(n, dtype=np.int64) * S, n * S, keys, kidx)
    assert r["checked"] == n and r["mismatches"] == 0, r
    # oracle-produced datagrams opened on the GPU
    lo, k = n // 2 + 7, 1 << 16
    rng = np.random.default_rng(2)
    host_pt = rng.integers(0, 256, k * S, dtype=np.uint8)
    od = np.zeros(k, DESC)
    od["src_off"] = od["dst_off"] = np.arange(k, dtype=np.int64) * S
    od["counter"] = rng.integers(0, 2**63, k, dtype=np.uint64)
    od["len"] = P
    host_wire = np.zeros(k * S, np.uint8)
    assert (o.seal_batch(od, keys, kidx, host_pt, host_wire) == 0).all()
    wire[lo * S:(lo + k) * S] = to_dev(torch, host_wire)
    back.zero_()
    st.fill_(-1)
    gpu.open_strided(n, P + 32, 0, wire, S, back, S, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    got = back[lo * S:(lo + k) * S].cpu().numpy().reshape(k, S)
    assert np.array_equal(got[:, :P], host_pt.reshape(k, S)[:, :P])
    assert torch.equal(back.view(n, S)[:lo, :P], pt.view(n, S)[:lo, :P])


@pytest.mark.parametrize("layout", ["slots_padded", "neptun"])
def test_config2_full_size_bench_layouts(torch_cuda, gpu, layout):
    """1M x 1350 B in bench.py's two config-2 layouts, full size:
    slots_padded -- plaintext at slot+16 sealed to a separate wire buffer and opened
      back to slot+16 with slot padding on (the headline line's layout): every
      seal output zero-filled from byte 1382 to its slot's line end (1408), every
      open output's 16 head bytes and bytes 1366..1407 zeroed, nothing else;
    neptun -- seal in place (device/mod.rs:1297-1337), open into fresh slots at
      offset 0 (device/mod.rs:1140-1148, the text grid), no padding: the bytes of
      the open slots past the plaintext untouched.
    Both: all statuses Ok, open(seal(x)) == x, every datagram equal to the oracle's
    (chunked host comparison)."""
    torch = torch_cuda
    n, P, S = 1 << 20, 1350, 1408
    keys = synth.keys(1)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    pt = synth.device_payloads(n, P, S, "cuda", offset=16)
    st_s = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    st_o = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    back = torch.full((n * S,), 0xCD, dtype=torch.uint8, device="cuda")
    if layout == "slots_padded":
        wire = torch.full((n * S,), 0xAB, dtype=torch.uint8, device="cuda")
        gpu.set_slot_padding(True)
        try:
            gpu.seal_strided(n, P, 0, 0, pt.data_ptr() + 16, S, wire, S, st_s)
            gpu.open_strided(n, P + 32, 0, wire, S, back.data_ptr() + 16, S, st_o)
            torch.cuda.synchronize()
        finally:
            gpu.set_slot_padding(False)
        o_off = 16
        w2, b2 = wire.view(n, S), back.view(n, S)
        assert bool((w2[:, P + 32:] == 0).all()), "seal: slot padding past the datagram"
        assert bool((b2[:, :16] == 0).all()) and bool((b2[:, 16 + P:] == 0).all()), "open: slot padding"
    else:
        wire = pt.clone()  # the TUN buffers, sealed in place
        gpu.seal_strided(n, P, 0, 0, wire.data_ptr() + 16, S, wire, S, st_s)
        gpu.open_strided(n, P + 32, 0, wire, S, back, S, st_o)
        torch.cuda.synchronize()
        o_off = 0
        b2 = back.view(n, S)
        assert bool((b2[:, P:] == 0xCD).all()), "open: bytes past the plaintext written"
        assert bool((wire.view(n, S)[:, P + 32:] == pt.view(n, S)[:, P + 32:]).all()), \
            "in-place seal: bytes past the datagram written"
    assert int((st_s != 0).sum()) == 0 and int((st_o != 0).sum()) == 0
    assert torch.equal(back.view(n, S)[:, o_off:o_off + P], pt.view(n, S)[:, 16:16 + P])
    from oracle_chunks import seal_matches_oracle
    descs = np.zeros(n, DESC)
    descs["src_off"] = np.arange(n, dtype=np.int64) * S + 16
    descs["dst_off"] = np.arange(n, dtype=np.int64) * S
    descs["counter"] = np.arange(n, dtype=np.uint64)
    descs["len"] = P
    r = seal_matches_oracle(pt, wire, descs, np.arange(n, dtype=np.int64) * S, n * S, keys,
                            np.array([synth.RECEIVER_IDX], np.uint32))
    assert r["checked"] == n and r["mismatches"] == 0, r


# ---------------------------------------------------------------------------
# mixed-length scheduling (BASELINE config 3) and per-peer keys (config 4)
# ---------------------------------------------------------------------------
def rounds_of(lens):
    return (lens.astype(np.int64) + 127) // 128


def test_plan_batch_is_a_length_sorted_permutation(torch_cuda, gpu):
    torch = torch_cuda
    from tools import workloads
    b = workloads.config3(1000, "cuda", seed=11)
    gpu.plan_batch(True, b.d_seal, b.n, b.order, b.scratch)
    torch.cuda.synchronize()
    order = b.order.cpu().numpy().astype(np.int64)
    assert np.array_equal(np.sort(order), np.arange(b.n))
    r = rounds_of(b.sizes[order] + 32)
    assert (np.diff(r) <= 0).all(), "longest packets first"
    # inside a bin the permutation keeps index order: deterministic
    for rr in np.unique(r):
        assert (np.diff(order[r == rr]) > 0).all()
    b.order.zero_()
    gpu.plan_batch(True, b.d_seal, b.n, b.order, b.scratch)
    torch.cuda.synchronize()
    assert np.array_equal(b.order.cpu().numpy().astype(np.int64), order)


@pytest.mark.parametrize("n", [1, 63, 4097, 256 * 4096 + 12345])
def test_plan_batch_equals_stable_sort_by_rounds(torch_cuda, gpu, n):
    """The permutation is exactly a stable sort by round count, longest first
    (ties keep index order), whatever the tiling: sizes with one partial chunk per
    tile up to several 4096-descriptor chunks per tile.  Lengths cover the clamp
    (>= 255 rounds share one bin) and zero."""
    torch = torch_cuda
    from neptun_amd.gpu import DESC_DTYPE
    rng = np.random.default_rng(n)
    lens = rng.choice(np.array([0, 1, 64, 96, 97, 256, 576, 1350, 8900, 40000, 70000], np.uint32), n)
    for seal, extra in ((True, 32), (False, 0)):
        d = np.zeros(n, DESC_DTYPE)
        d["len"] = lens
        descs = torch.from_numpy(d.view(np.uint8)).to("cuda")
        order = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        scratch = torch.empty(256 * 256, dtype=torch.int32, device="cuda")
        gpu.plan_batch(seal, descs, n, order, scratch)
        torch.cuda.synchronize()
        got = order.cpu().numpy().astype(np.int64)
        rounds = np.minimum((lens.astype(np.int64) + extra + 127) // 128, 255)
        want = np.argsort(-rounds, kind="stable")
        assert np.array_equal(got, want), (seal, n)


@pytest.mark.parametrize("ordered", [True, False])
def test_mixed_mtu_batch_matches_oracle(torch_cuda, gpu, ordered):
    torch = torch_cuda
    from tools import workloads
    b = workloads.config3(2000, "cuda", seed=12)
    keys = synth.keys(1, seed=77)
    kidx = np.array([0xBEEF], np.uint32)
    gpu.set_keys(0, keys, kidx)
    if ordered:
        gpu.plan_batch(True, b.d_seal, b.n, b.order, b.scratch)
        gpu.seal_batch_ordered(b.d_seal, b.order, b.n, b.pt, b.wire, b.st_seal)
        gpu.open_batch_ordered(b.d_open, b.order, b.n, b.wire, b.out, b.st_open)
    else:
        gpu.seal_batch(b.d_seal, b.n, b.pt, b.wire, b.st_seal)
        gpu.open_batch(b.d_open, b.n, b.wire, b.out, b.st_open)
    torch.cuda.synchronize()
    assert int((b.st_seal != 0).sum()) == 0 and int((b.st_open != 0).sum()) == 0
    src = b.pt.cpu().numpy()
    want = np.zeros_like(src)
    assert (o.seal_batch(b.seal_host, keys, kidx, src, want) == 0).all()
    assert np.array_equal(b.wire.cpu().numpy(), want)
    assert b.round_trip_equal()


def test_per_peer_keys_match_oracle(torch_cuda, gpu):
    """Config 4 shape at reduced size: 512 peers x 32 packets, keys looked up per lane."""
    torch = torch_cuda
    from tools import workloads
    peers, per = 512, 32
    b = workloads.config4(peers, per, 1350, "cuda", seed=13)
    keys = synth.keys(peers, seed=99)
    kidx = (np.arange(peers, dtype=np.uint32) * 2654435761).astype(np.uint32)
    gpu.set_keys(0, keys, kidx)
    gpu.seal_batch(b.d_seal, b.n, b.pt, b.wire, b.st_seal)
    gpu.open_batch(b.d_open, b.n, b.wire, b.out, b.st_open)
    torch.cuda.synchronize()
    assert int((b.st_seal != 0).sum()) == 0 and int((b.st_open != 0).sum()) == 0
    src = b.pt.cpu().numpy()
    want = np.zeros_like(src)
    assert (o.seal_batch(b.seal_host, keys, kidx, src, want) == 0).all()
    assert np.array_equal(b.wire.cpu().numpy(), want)
    # per-peer counters 0..per-1 made it into the headers
    w = b.wire.cpu().numpy()
    ctr = np.array([int.from_bytes(w[x + 8:x + 16].tobytes(), "little") for x in b.offs])
    peer = b.seal_host["key_slot"]
    for pr in range(0, peers, 97):
        assert sorted(ctr[peer == pr]) == list(range(per))
    assert b.round_trip_equal()


def test_config4_full_size_per_peer(torch_cuda, gpu):
    """BASELINE config 4 at full size: 4096 peers x 4096 packets (16.8M x 1350 B, keys
    per lane from the 4096-slot table): statuses, round trip, every peer's counters
    exactly 0..4095 and its receiver index in its headers, and every datagram equal to
    the oracle's (chunked host comparison over the 22.6 GB batch)."""
    torch = torch_cuda
    from tools import workloads
    peers = per = 4096
    b = workloads.config4(peers, per, 1350, "cuda", seed=17)
    keys = synth.keys(peers, seed=5)
    kidx = (np.arange(peers, dtype=np.uint32) * 2246822519).astype(np.uint32)
    gpu.set_keys(0, keys, kidx)
    gpu.seal_batch(b.d_seal, b.n, b.pt, b.wire, b.st_seal)
    gpu.open_batch(b.d_open, b.n, b.wire, b.out, b.st_open)
    torch.cuda.synchronize()
    assert int((b.st_seal != 0).sum()) == 0 and int((b.st_open != 0).sum()) == 0
    assert b.round_trip_equal(chunk=1 << 16)
    # header counters: (peer, counter) pairs are exactly peers x 0..per-1
    offs = torch.from_numpy(b.offs).cuda()
    ctr = torch.zeros(b.n, dtype=torch.int64, device="cuda")
    for j in range(8):
        ctr |= b.wire[offs + 8 + j].to(torch.int64) << (8 * j)
    peer = torch.from_numpy(b.seal_host["key_slot"].astype(np.int64)).cuda()
    key = torch.sort(peer * per + ctr).values
    assert torch.equal(key, torch.arange(b.n, dtype=torch.int64, device="cuda"))
    # every header's receiver index is its peer's key_index (no slot mix-up)
    ridx = torch.zeros(b.n, dtype=torch.int64, device="cuda")
    for j in range(4):
        ridx |= b.wire[offs + 4 + j].to(torch.int64) << (8 * j)
    want_ridx = torch.from_numpy(kidx.astype(np.int64)).cuda()[peer]
    assert torch.equal(ridx, want_ridx)
    del key, ctr, offs, peer, ridx, want_ridx
    # every datagram against the oracle (chunked host comparison)
    from oracle_chunks import seal_matches_oracle
    r = seal_matches_oracle(b.pt, b.wire, b.seal_host, b.offs, b.total, keys, kidx)
    assert r["checked"] == b.n and r["mismatches"] == 0, r


def test_config3_full_size_round_trip(torch_cuda, gpu):
    """BASELINE config 3 at full size (1.31M packets): statuses, round trip, every datagram
    equal to the oracle's (chunked host comparison)."""
    torch = torch_cuda
    from tools import workloads
    b = workloads.config3(1 << 18, "cuda")
    keys = synth.keys(1)
    kidx = np.array([synth.RECEIVER_IDX], np.uint32)
    gpu.set_keys(0, keys, kidx)
    gpu.plan_batch(True, b.d_seal, b.n, b.order, b.scratch)
    gpu.seal_batch_ordered(b.d_seal, b.order, b.n, b.pt, b.wire, b.st_seal)
    gpu.open_batch_ordered(b.d_open, b.order, b.n, b.wire, b.out, b.st_open)
    torch.cuda.synchronize()
    assert int((b.st_seal != 0).sum()) == 0 and int((b.st_open != 0).sum()) == 0
    assert b.round_trip_equal()
    from oracle_chunks import seal_matches_oracle
    r = seal_matches_oracle(b.pt, b.wire, b.seal_host, b.offs, b.total, keys, kidx)
    assert r["checked"] == b.n and r["mismatches"] == 0, r


# ---------------------------------------------------------------------------
# host-resident pipeline (pinned staging + overlapped hipMemcpyAsync)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("depth,chunk", [(3, 1 << 20), (2, 5 << 20)])
def test_host_pipe_matches_device_path(torch_cuda, gpu, depth, chunk):
    torch = torch_cuda
    import neptun_amd
    n, P = 10007, 1350           # not a multiple of the chunk's packet count
    S_host = 1392                # a host layout that is not the device slot layout
    keys = synth.keys(1, seed=5)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    pipe = neptun_amd.GpuPipe(gpu, chunk_bytes=chunk, depth=depth)
    pt = torch.randint(0, 256, (n * S_host,), dtype=torch.uint8).pin_memory()
    wire = torch.zeros(n * S_host, dtype=torch.uint8).pin_memory()
    back = torch.zeros(n * S_host, dtype=torch.uint8).pin_memory()
    st = torch.full((n,), -1, dtype=torch.int32).pin_memory()
    pipe.seal_strided(n, P, 0, 1234, pt, S_host, wire, S_host, st)
    assert int((st != 0).sum()) == 0
    # reference: oracle on a sample, device strided path on all
    w = wire.numpy().reshape(n, S_host)
    p = pt.numpy().reshape(n, S_host)
    for i in (0, 1, 4095, 4096, n - 1):
        assert w[i, :P + 32].tobytes() == o.format_packet_data(
            keys[0].tobytes(), synth.RECEIVER_IDX, 1234 + i, p[i, :P].tobytes())
    d_pt = pt.cuda()
    d_wire = torch.zeros(n * S_host, dtype=torch.uint8, device="cuda")
    gpu.seal_strided(n, P, 0, 1234, d_pt, S_host, d_wire, S_host)
    torch.cuda.synchronize()
    dw = d_wire.cpu().numpy().reshape(n, S_host)
    assert np.array_equal(w[:, :P + 32], dw[:, :P + 32])
    assert not w[:, P + 32:].any()   # only packet bytes are written back
    st.fill_(-1)
    pipe.open_strided(n, P + 32, 0, wire, S_host, back, S_host, st)
    assert int((st != 0).sum()) == 0
    assert np.array_equal(back.numpy().reshape(n, S_host)[:, :P], p[:, :P])
    pipe.close()


@pytest.mark.parametrize("out_off", [16, 0])
@pytest.mark.parametrize("P", list(range(0, 70)) + [127, 128, 129, 240, 255, 256, 257, 1000, 1349,
                                                   1350, 1351, 1407, 1500, 8900])
def test_strided_every_tail_shape(torch_cuda, gpu, P, out_off):
    """Uniform strided kernel (+ its one-wave tail launch) at lengths covering every
    partial-chunk size 0..15 on both sides: wire bytes equal the oracle's, nothing
    is written outside each packet (guard bytes), open restores the plaintext.
    out_off = where open's plaintext sits in its 128-byte-multiple slot: 16 (the
    wire run grid) or 0 (slot-aligned plaintext: the text run grid kernel)."""
    torch = torch_cuda
    n = 130  # two full uniform waves + a 2-packet tail wave
    S = synth.round_up(P + 32 + 16, 128)
    keys = synth.keys(1, seed=P + 1)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    rng = np.random.default_rng(P)
    src = rng.integers(0, 256, n * S, dtype=np.uint8)
    pt = to_dev(torch, src)
    wire = torch.full((n * S,), 0xAB, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.seal_strided(n, P, 0, 5 + P, pt.data_ptr() + 16, S, wire, S, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    descs = np.zeros(n, DESC)
    descs["src_off"] = np.arange(n) * S + 16
    descs["dst_off"] = np.arange(n) * S
    descs["counter"] = 5 + P + np.arange(n, dtype=np.uint64)
    descs["len"] = P
    want = np.full(n * S, 0xAB, np.uint8)
    assert (o.seal_batch(descs, keys, np.array([synth.RECEIVER_IDX], np.uint32), src, want) == 0).all()
    assert np.array_equal(wire.cpu().numpy(), want)  # includes the guard bytes past P + 32
    back = torch.full((n * S,), 0xCD, dtype=torch.uint8, device="cuda")
    st.fill_(-1)
    assert back.data_ptr() % 128 == 0 and S % 128 == 0
    gpu.open_strided(n, P + 32, 0, wire, S, back.data_ptr() + out_off, S, st)
    torch.cuda.synchronize()
    assert (st == 0).all()
    got = back.cpu().numpy().reshape(n, S)
    assert np.array_equal(got[:, out_off:out_off + P], src.reshape(n, S)[:, 16:16 + P])
    assert (got[:, :out_off] == 0xCD).all() and (got[:, out_off + P:] == 0xCD).all()


def test_device_routing_then_open_matches_oracle(torch_cuda, gpu):
    """Raw inbound datagrams -> wg_gpu_route_batch (receiver_idx -> key slot on the device,
    device/mod.rs:1022-1024 + noise/mod.rs:550-556) -> open: same plaintext and status as
    the oracle; unknown receivers are NoCurrentSession, non-DATA messages InvalidPacket."""
    import random
    from neptun_amd.gpu import KEY_SLOT_INVALID_PACKET, KEY_SLOT_NO_SESSION
    torch = torch_cuda
    rng = random.Random(11)
    n_sess, first = 40, 1000
    locals_ = rng.sample(range(1, 2**32), n_sess)
    keys = np.frombuffer(rng.randbytes(32 * n_sess), np.uint8).reshape(n_sess, 32)
    gpu.set_keys(first, keys, np.array(locals_, np.uint32))
    gpu.route_set(np.array(locals_, np.uint32), np.arange(first, first + n_sess, dtype=np.uint32))
    items, want_slot, want = [], [], []
    for _ in range(600):
        r = rng.random()
        j = rng.randrange(n_sess)
        P = rng.choice([0, 1, 15, 16, 17, 64, 576, 1350, rng.randrange(0, 1500)])
        pt = rng.randbytes(P)
        if r < 0.8:
            d = o.format_packet_data(bytes(keys[j]), locals_[j], rng.getrandbits(64), pt)
            if rng.random() < 0.05:
                d = bytearray(d)
                d[-1] ^= 1
                d = bytes(d)
            items.append(d)
            want_slot.append(first + j)
            want.append(o.receive_packet_data(bytes(keys[j]), locals_[j], d))
        elif r < 0.9:
            unknown = rng.getrandbits(32)
            while unknown in locals_:
                unknown = rng.getrandbits(32)
            items.append(o.format_packet_data(bytes(keys[j]), unknown, 1, pt))
            want_slot.append(KEY_SLOT_NO_SESSION)
            want.append((14, b""))
        else:
            kind = rng.randrange(3)
            d = (struct_le(1) + rng.randbytes(144) if kind == 0 else
                 struct_le(4) + rng.randbytes(rng.randrange(0, 28)) if kind == 1 else
                 struct_le(7) + rng.randbytes(60))
            items.append(d)
            want_slot.append(KEY_SLOT_INVALID_PACKET)
            want.append((13, b""))
    src, offs = pack(items)
    descs = np.zeros(len(items), DESC)
    descs["src_off"] = offs
    descs["dst_off"] = np.array(offs) + 16
    descs["len"] = [len(x) for x in items]
    descs["key_slot"] = 7  # overwritten by the router
    d_descs = to_dev(torch, descs.view(np.uint8))
    d_src = to_dev(torch, src)
    gpu.route_batch(d_descs, len(items), d_src)
    torch.cuda.synchronize()
    routed = d_descs.cpu().numpy().view(DESC)
    assert list(routed["key_slot"]) == want_slot
    d_dst = torch.zeros(len(src), dtype=torch.uint8, device="cuda")
    d_st = torch.full((len(items),), -1, dtype=torch.int32, device="cuda")
    gpu.open_batch(d_descs, len(items), d_src, d_dst, d_st)
    torch.cuda.synchronize()
    st, out = d_st.cpu().numpy(), d_dst.cpu().numpy()
    for i, (ws, wpt) in enumerate(want):
        assert st[i] == ws, (i, st[i], ws)
        if ws == 0:
            assert out[offs[i] + 16:offs[i] + 16 + len(wpt)].tobytes() == wpt


def struct_le(v):
    return int(v).to_bytes(4, "little")


def test_jumbo_and_extreme_lengths_match_oracle(torch_cuda, gpu):
    """Descriptor path at the length extremes: empty, sub-chunk, MTU, jumbo and the
    largest IPv4 datagram payload (the planner clamps >= 255 rounds into one bin)."""
    torch = torch_cuda
    rng = np.random.default_rng(3)
    sizes = [0, 1, 15, 16, 17, 8900, 9000, 32768, 65503, 65535 - 32]
    keys = synth.keys(2, seed=4)
    gpu.set_keys(0, keys, np.array([11, 22], np.uint32))
    items = [rng.integers(0, 256, s, np.uint8).tobytes() for s in sizes]
    src, offs = pack(items, pad=48)
    descs = np.zeros(len(items), DESC)
    for i, s in enumerate(sizes):
        descs[i] = (offs[i], offs[i], (1 << 63) + i, s, i & 1)
    # seal into a separate buffer at the same offsets (+16 B headroom per slot)
    out, st = run_desc(torch, gpu, True, descs, src, len(src) + 64)
    assert (st == 0).all()
    want = np.zeros_like(out)
    assert (o.seal_batch(descs, keys, np.array([11, 22], np.uint32), src, want) == 0).all()
    for i, s in enumerate(sizes):
        assert out[offs[i]:offs[i] + s + 32].tobytes() == want[offs[i]:offs[i] + s + 32].tobytes(), s
    opn = descs.copy()
    opn["len"] = np.array(sizes) + 32
    opn["dst_off"] = np.array(offs) + 16
    back, st = run_desc(torch, gpu, False, opn, out, len(out) + 64)
    assert (st == 0).all()
    for i, s in enumerate(sizes):
        assert back[offs[i] + 16:offs[i] + 16 + s].tobytes() == items[i]


def test_argument_validation_fails_loudly(torch_cuda, gpu):
    """Bad arguments are rejected by the ABI (no launch) with a message."""
    import neptun_amd
    torch = torch_cuda
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with pytest.raises(neptun_amd.NeptunGpuError, match="16-byte aligned"):
        gpu.seal_strided(64, 100, 0, 0, buf.data_ptr() + 4, 256, buf, 256)
    with pytest.raises(neptun_amd.NeptunGpuError, match="bad key slot"):
        gpu.seal_strided(64, 100, 1 << 20, 0, buf, 256, buf, 256)
    # slots that would overlap their neighbours, and strides past the 32-bit
    # buffer-offset reach of the uniform kernels
    with pytest.raises(neptun_amd.NeptunGpuError, match="exceeds its stride"):
        gpu.seal_strided(64, 240, 0, 0, buf, 256, buf, 256)  # datagram 272 > 256
    with pytest.raises(neptun_amd.NeptunGpuError, match="exceeds its stride"):
        gpu.open_strided(64, 300, 0, buf, 256, buf, 512)  # datagram 300 > 256
    with pytest.raises(neptun_amd.NeptunGpuError, match="stride too large"):
        gpu.seal_strided(64, 100, 0, 0, buf, 64 << 20, buf, 256)
    with pytest.raises(neptun_amd.NeptunGpuError, match="slot range"):
        gpu.set_keys(4095, synth.keys(2), np.array([1, 2], np.uint32))
    with pytest.raises(neptun_amd.NeptunGpuError, match="duplicate receiver"):
        gpu.route_set(np.array([5, 5], np.uint32), np.array([0, 1], np.uint32))
    with pytest.raises(neptun_amd.NeptunGpuError, match="outside the key table"):
        gpu.route_set(np.array([5], np.uint32), np.array([1 << 20], np.uint32))


def test_persistent_grid_partial_group_dropped_lanes(torch_cuda, gpu):
    """Strided batch larger than one pass of the persistent grid (2 workgroups
    per CU x 512 packets), ending in a partial workgroup group and a tail wave;
    open with dropped lanes (bad type, wrong index) and forged tags scattered
    over the waves, so the phase-locked path runs with dead lanes in many
    workgroups.  Statuses, stored bytes and zeroing follow session.rs:265-302
    and noise/mod.rs:139-199 (oracle spot checks)."""
    torch = torch_cuda
    n, P, S = 512 * 520 + 64 * 3 + 17, 1350, 1408
    keys = synth.keys(1)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    pt = synth.device_payloads(n, P, S, "cuda", seed=11)
    wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    back = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    base = 0xFFFF_FF00  # counters cross 2^32 inside the batch
    gpu.seal_strided(n, P, 0, base, pt, S, wire, S, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    rng = np.random.default_rng(5)
    bad_type = rng.choice(n, 300, replace=False)
    rest = np.setdiff1d(np.arange(n), bad_type)
    wrong_idx = rng.choice(rest, 300, replace=False)
    rest = np.setdiff1d(rest, wrong_idx)
    forged = rng.choice(rest, 300, replace=False)
    w = wire.view(n, S)
    w[torch.from_numpy(bad_type).cuda(), 0] = 2
    w[torch.from_numpy(wrong_idx).cuda(), 4] ^= 1
    w[torch.from_numpy(forged).cuda(), P + 20] ^= 0x80   # a tag byte
    gpu.open_strided(n, P + 32, 0, wire, S, back, S, st)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    want = np.zeros(n, np.int32)
    want[bad_type] = 13   # InvalidPacket
    want[wrong_idx] = 5   # WrongIndex
    want[forged] = 10     # InvalidAeadTag
    assert np.array_equal(s, want)
    b = back.view(n, S)
    p = pt.view(n, S)
    ok = torch.from_numpy(np.flatnonzero(want == 0)).cuda()
    assert torch.equal(b[ok, :P], p[ok, :P])
    # dropped packets store nothing; forged ones are zeroed (ring open_in_place)
    assert int(b[torch.from_numpy(bad_type).cuda()].abs().sum()) == 0
    assert int(b[torch.from_numpy(wrong_idx).cuda()].abs().sum()) == 0
    assert int(b[torch.from_numpy(forged).cuda(), :P].abs().sum()) == 0
    # oracle spot checks of the sealed bytes across groups, waves and the tail
    rows = np.concatenate([np.arange(0, n, 4999), [n - 18, n - 17, n - 1]])
    wr = w[torch.from_numpy(rows).cuda()].cpu().numpy()
    pr = p[torch.from_numpy(rows).cuda()].cpu().numpy()
    for r, wrow, prow in zip(rows, wr, pr):
        if r in bad_type or r in wrong_idx or r in forged:
            continue
        want_w = o.format_packet_data(keys[0].tobytes(), synth.RECEIVER_IDX, base + int(r), prow[:P].tobytes())
        assert wrow[:P + 32].tobytes() == want_w


@pytest.mark.parametrize("P,out_off,src_stride,dst_stride", [
    (1350, 16, 1408, 1408), (1350, 0, 1408, 1408), (1290, 16, 1408, 1408), (64, 16, 128, 128),
    (0, 16, 128, 128), (127, 0, 256, 256), (1392, 16, 1536, 1408), (1400, 16, 1536, 1408)])
def test_strided_slot_padding(torch_cuda, gpu, P, out_off, src_stride, dst_stride):
    """wg_gpu_ctx_set_slot_padding: outputs are unchanged; from each output's end to the
    next 128-byte boundary of its slot the bytes are zero, and for open on the wire grid
    the 16 slot bytes before the plaintext (uniform waves; the one-wave tail launch does
    not pad); nothing else is written; no padding where the boundary would leave the
    slot (1400 / 1408)."""
    torch = torch_cuda
    n = 130
    keys = synth.keys(1, seed=P + 7)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    rng = np.random.default_rng(P + 1)
    S = src_stride
    src = rng.integers(0, 256, n * S, dtype=np.uint8)
    pt = to_dev(torch, src)
    wire = torch.full((n * S,), 0xAB, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.set_slot_padding(True)
    try:
        gpu.seal_strided(n, P, 0, 3, pt.data_ptr() + 16, S, wire, S, st)
        torch.cuda.synchronize()
        assert (st == 0).all()
        descs = np.zeros(n, DESC)
        descs["src_off"] = np.arange(n) * S + 16
        descs["dst_off"] = np.arange(n) * S
        descs["counter"] = 3 + np.arange(n, dtype=np.uint64)
        descs["len"] = P
        want = np.full(n * S, 0xAB, np.uint8)
        assert (o.seal_batch(descs, keys, np.array([synth.RECEIVER_IDX], np.uint32), src, want) == 0).all()
        want = want.reshape(n, S)
        W = P + 32
        end = -(-W // 128) * 128
        if end <= S:
            want[:n & ~63, W:end] = 0  # seal's slot = [dst, dst + stride)
        assert np.array_equal(wire.cpu().numpy().reshape(n, S), want)
        D = dst_stride
        back = torch.full((n * D + 64,), 0xCD, dtype=torch.uint8, device="cuda")
        st.fill_(-1)
        gpu.open_strided(n, W, 0, wire, S, back.data_ptr() + out_off, D, st)
        torch.cuda.synchronize()
        assert (st == 0).all()
        got = back.cpu().numpy()
        exp = np.full(n * D + 64, 0xCD, np.uint8)  # (outputs may straddle D-rows: flat)
        # the run grid's origin: dst (text grid, slot-aligned plaintext) or dst - 16
        origin = out_off if out_off % 128 == 0 else out_off - 16
        end = origin + -(-(out_off - origin + P) // 128) * 128
        pad = origin % 128 == 0 and D % 128 == 0 and end - origin <= D
        rows = src.reshape(n, S)
        for i in range(n):
            exp[i * D + out_off:i * D + out_off + P] = rows[i, 16:16 + P]
            if pad and i < (n & ~63):
                exp[i * D + out_off + P:i * D + end] = 0
                exp[i * D + origin:i * D + out_off] = 0  # (wire grid: the slot's 16 head bytes)
        assert np.array_equal(got, exp)
    finally:
        gpu.set_slot_padding(False)


def test_one_context_from_two_threads(torch_cuda, gpu):
    """include/neptun_gpu.h: a context may be used from several host threads.  Two
    threads seal and open their own strided batches on their own streams, with
    different key slots, concurrently; both match the oracle."""
    import threading
    torch = torch_cuda
    keys = synth.keys(2, seed=77)
    idx = np.array([0x1234, 0x5678], np.uint32)
    gpu.set_keys(0, keys, idx)
    n, P, S = 4096 + 17, 1350, 1408
    results, errors = {}, []

    def worker(t):
        try:
            stream = torch.cuda.Stream()
            pt = synth.device_payloads(n, P, S, "cuda", seed=100 + t)
            wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
            back = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
            st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            for _ in range(20):
                gpu.seal_strided(n, P, t, 1000 * t, pt.data_ptr() + 16, S, wire, S, st, stream=stream)
                gpu.open_strided(n, P + 32, t, wire, S, back.data_ptr() + 16, S, st, stream=stream)
            stream.synchronize()
            results[t] = (pt, wire, back, st)
        except Exception as e:  # reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in (0, 1)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in (0, 1):
        pt, wire, back, st = results[t]
        assert int((st != 0).sum()) == 0
        assert torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P])
        for i in (0, 1, 63, 64, 2049, n - 1):
            row = pt.view(n, S)[i, 16:16 + P].cpu().numpy().tobytes()
            want = o.format_packet_data(keys[t].tobytes(), int(idx[t]), 1000 * t + i, row)
            assert wire.view(n, S)[i, :P + 32].cpu().numpy().tobytes() == want


def test_descriptor_wave_shapes_match_oracle(torch_cuda, gpu):
    """The descriptor kernels' wave-level forms -- waves whose live packets share one
    key slot (the SGPR-key form when built with WG_DESC_UNIFORM_KEY) or not, rounds
    every live packet fills (the full-round form) and rounds near that boundary
    (P = 128 r + 112 +- 1), waves with failed lanes (bad key slot, misaligned) beside
    live ones -- sealed and opened bit-exact against the oracle, with tampered
    datagrams rejected and zeroed."""
    torch = torch_cuda
    rng = np.random.default_rng(97)
    n_keys = 16
    keys = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, n_keys, dtype=np.uint64).astype(np.uint32)
    gpu.set_keys(0, keys, kidx)
    waves = 24  # 3 workgroups of 8 waves
    n = 64 * waves
    sizes = np.zeros(n, np.int64)
    slots = np.zeros(n, np.uint32)
    bound = [111, 112, 113, 239, 240, 241, 367, 368, 369, 1391, 1392, 1393]
    for w in range(waves):
        lo, kind = 64 * w, w % 4
        if kind == 0:      # one key, one length
            sizes[lo:lo + 64], slots[lo:lo + 64] = 1350, w % n_keys
        elif kind == 1:    # one key, lengths around the full-round boundaries
            sizes[lo:lo + 64] = rng.choice(bound, 64)
            slots[lo:lo + 64] = (w * 7) % n_keys
        elif kind == 2:    # mixed keys, long packets plus one empty and one tiny one
            sizes[lo:lo + 64] = rng.choice([1350, 8900, 2000], 64)
            sizes[lo + 5], sizes[lo + 40] = 0, 16
            slots[lo:lo + 64] = rng.integers(0, n_keys, 64)
        else:              # one key, but some lanes fail before the crypto
            sizes[lo:lo + 64] = rng.integers(0, 3000, 64)
            slots[lo:lo + 64] = 3
    payloads = synth.host_payloads(sizes, seed=98)
    src, soffs = pack(payloads)
    doffs, pos = [], 0
    for s in sizes:
        doffs.append(pos)
        pos = synth.round_up(pos + int(s) + 32, 16)
    descs = np.zeros(n, DESC)
    descs["src_off"] = soffs
    descs["dst_off"] = doffs
    descs["counter"] = rng.integers(0, 2**62, n, dtype=np.uint64)
    descs["len"] = sizes
    descs["key_slot"] = slots
    bad_slot = [64 * 3 + 2, 64 * 7 + 63, 64 * 11]
    misaligned = [64 * 3 + 9, 64 * 15 + 1]
    descs["key_slot"][bad_slot] = gpu.key_slots + 5  # past the context's key table
    descs["src_off"][misaligned] += 4
    valid = np.ones(n, bool)
    valid[bad_slot + misaligned] = False
    out, st = run_desc(torch, gpu, True, descs, src, pos + 64)
    assert (st[bad_slot] == 101).all() and (st[misaligned] == 100).all()
    want = np.zeros(pos + 64, np.uint8)
    wst = o.seal_batch(descs[valid], keys, kidx, src, want)
    assert (wst == 0).all() and (st[valid] == 0).all()
    assert np.array_equal(out, want), "sealed bytes differ from the oracle"
    # open the valid datagrams back, a few of them tampered
    vi = np.nonzero(valid)[0]
    d2 = np.zeros(len(vi), DESC)
    d2["src_off"] = np.array(doffs)[vi]
    d2["dst_off"] = np.array(soffs)[vi]
    d2["len"] = sizes[vi] + 32
    d2["key_slot"] = slots[vi]
    wire = out.copy()
    tampered = rng.choice(len(vi), 12, replace=False)
    for t in tampered:
        L = int(sizes[vi[t]]) + 32
        wire[int(d2["src_off"][t]) + int(rng.integers(16, L))] ^= 0x40
    back, st2 = run_desc(torch, gpu, False, d2, wire, len(src))
    want2 = np.zeros(len(src), np.uint8)
    wst2 = o.open_batch(d2, keys, kidx, wire, want2)
    assert (st2 == wst2).all(), (st2[tampered], wst2[tampered])
    assert (st2[tampered] == 10).all()
    for t in range(len(vi)):  # plaintext bytes (tampered ones zeroed, like ring)
        a, P = int(d2["dst_off"][t]), int(sizes[vi[t]])
        if t in set(tampered.tolist()):
            assert not back[a:a + P].any()
        else:
            assert np.array_equal(back[a:a + P], want2[a:a + P]) and np.array_equal(back[a:a + P], src[a:a + P])


@pytest.mark.parametrize("P,ss,sd,n,base,breaks", [
    (1350, 1408, 1408, 512 * 3 + 64 * 3 + 17, (0, 0), ()),   # config 4's slots; partial last group
    (64, 96, 96, 1024, (48, 16), ()),                          # tight strides, lines not 128-aligned
    (0, 32, 32, 512, (0, 0), ()),                              # empty payloads
    (1000, 1152, 1040, 1536, (16, 0), (600,)),                 # unequal strides; group 1 not affine
    (8900, 8960, 8960, 576, (0, 128), ()),                     # jumbo
])
def test_affine_descriptor_groups_match_oracle(torch_cuda, gpu, P, ss, sd, n, base, breaks):
    """Descriptor batches whose workgroups hold one length at constant slot strides
    run the uniform geometry with per-packet keys (WG_DESC_AFFINE): sealed and opened
    bit-exact against the oracle over the whole destination (no byte outside a packet
    written), beside groups that do not qualify (a partial last group, a group with
    one packet out of place) and with open's failures inside affine groups (tampered
    ciphertext zeroed, wrong receiver index, wrong message type)."""
    torch = torch_cuda
    rng = np.random.default_rng(P + n)
    n_keys = 64
    keys = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, n_keys, dtype=np.uint64).astype(np.uint32)
    gpu.set_keys(0, keys, kidx)
    sizes = np.full(n, P, np.int64)
    payloads = synth.host_payloads(sizes, seed=P + 7)
    soffs = base[0] + ss * np.arange(n, dtype=np.int64)
    doffs = base[1] + sd * np.arange(n, dtype=np.int64)
    for b in breaks:  # swap two packets' wire slots: that workgroup is not affine
        doffs[b], doffs[b + 1] = doffs[b + 1], doffs[b]
    src = np.zeros(int(soffs[-1]) + ss + 64, np.uint8)
    for i in range(n):
        src[soffs[i]:soffs[i] + P] = np.frombuffer(payloads[i], np.uint8)
    dst_size = int(doffs.max()) + sd + 64
    descs = np.zeros(n, DESC)
    descs["src_off"] = soffs
    descs["dst_off"] = doffs
    descs["counter"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    descs["counter"][:3] = [2**32 - 1, 2**32, 2**64 - 1]
    descs["len"] = sizes
    descs["key_slot"] = rng.integers(0, n_keys, n).astype(np.uint32)
    out, st = run_desc(torch, gpu, True, descs, src, dst_size)
    want = np.zeros(dst_size, np.uint8)
    wst = o.seal_batch(descs, keys, kidx, src, want)
    assert (wst == 0).all() and (st == 0).all(), np.unique(st)
    assert np.array_equal(out, want), "sealed bytes differ from the oracle"
    # open them back, with failures inside the (affine) first group
    d2 = np.zeros(n, DESC)
    d2["src_off"] = doffs
    d2["dst_off"] = soffs
    d2["len"] = sizes + 32
    d2["key_slot"] = descs["key_slot"]
    wire = out.copy()
    tampered, wrong_idx, wrong_type = [3, 200], [77], [130]
    for t in tampered:
        wire[int(doffs[t]) + 16 + int(rng.integers(0, P + 16))] ^= 0x10
    for t in wrong_idx:
        wire[int(doffs[t]) + 4] ^= 0x01
    for t in wrong_type:
        wire[int(doffs[t])] = 1
    back, st2 = run_desc(torch, gpu, False, d2, wire, len(src))
    want2 = np.zeros(len(src), np.uint8)
    wst2 = o.open_batch(d2, keys, kidx, wire, want2)
    assert (st2 == wst2).all(), [(i, st2[i], wst2[i]) for i in np.nonzero(st2 != wst2)[0][:8]]
    assert (st2[tampered] == 10).all() and (st2[wrong_idx] != 0).all() and (st2[wrong_type] != 0).all()
    assert np.array_equal(back, want2), "opened bytes differ from the oracle"
    ok = np.ones(n, bool)
    ok[tampered + wrong_idx + wrong_type] = False
    for i in np.nonzero(ok)[0][:: max(1, n // 97)]:
        assert np.array_equal(back[soffs[i]:soffs[i] + P], src[soffs[i]:soffs[i] + P])


@pytest.fixture(scope="module")
def gpu1(torch_cuda):
    """A single-slot context: its descriptor launches take the SGPR-key forms."""
    from neptun_amd import GpuContext
    ctx = GpuContext(0, key_slots=1)
    ctx.set_xlane_lanes(0)  # (the throughput forms, like the module's other tests)
    yield ctx
    ctx.close()


@pytest.mark.parametrize("form", ["mixed", "ordered", "affine"])
def test_single_slot_context_forms_match_oracle(torch_cuda, gpu1, form):
    """Descriptor batches on a one-slot context (aead_desc_*_key1_kernel: the key
    loaded once per kernel): unordered mixed lengths, the plan's ordered launch,
    and affine groups -- sealed and opened bit-exact against the oracle, with
    packets naming other slots failing with BAD_KEY_SLOT (open: the invalid and
    no-session markers keep their statuses), tampered datagrams rejected and
    zeroed, and a wrong receiver index refused."""
    torch = torch_cuda
    rng = np.random.default_rng({"mixed": 5, "ordered": 6, "affine": 7}[form])
    keys = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    kidx = np.array([0x5EED1234], np.uint32)
    gpu1.set_keys(0, keys, kidx)
    n = 512 * 4 + 200
    if form == "affine":
        P, S = 1350, 1408
        sizes = np.full(n, P, np.int64)
        soffs = S * np.arange(n, dtype=np.int64)
        doffs = soffs.copy()
        src = np.zeros(S * n + 64, np.uint8)
        for i, p in enumerate(synth.host_payloads(sizes, seed=8)):
            src[soffs[i]:soffs[i] + P] = np.frombuffer(p, np.uint8)
        dst_size = S * n + 64
    else:
        sizes = rng.choice([0, 1, 64, 255, 1350, 4000, 8900], n)
        src, soffs = pack(synth.host_payloads(sizes, seed=9))
        soffs = np.array(soffs, np.int64)
        doffs, pos = np.zeros(n, np.int64), 0
        for i in rng.permutation(n):
            doffs[i] = pos
            pos = synth.round_up(pos + int(sizes[i]) + 32, 16)
        dst_size = pos + 64
    descs = np.zeros(n, DESC)
    descs["src_off"], descs["dst_off"], descs["len"] = soffs, doffs, sizes
    descs["counter"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    bad = [] if form == "affine" else [7, 600, 1500]
    if bad:
        descs["key_slot"][bad] = [1, 5, 2**31]
    valid = np.ones(n, bool)
    valid[bad] = False

    def launch(seal, d, src_b, size):
        d_descs = to_dev(torch, d.view(np.uint8))
        d_src = to_dev(torch, src_b)
        d_dst = torch.zeros(max(size, 16), dtype=torch.uint8, device="cuda")
        d_st = torch.full((len(d),), -1, dtype=torch.int32, device="cuda")
        if form == "ordered":
            order = torch.zeros(len(d), dtype=torch.int32, device="cuda")
            scratch = torch.zeros(262144 // 4, dtype=torch.int32, device="cuda")
            gpu1.plan_batch(seal, d_descs, len(d), order, scratch)
            (gpu1.seal_batch_ordered if seal else gpu1.open_batch_ordered)(
                d_descs, order, len(d), d_src, d_dst, d_st)
        else:
            (gpu1.seal_batch if seal else gpu1.open_batch)(d_descs, len(d), d_src, d_dst, d_st)
        torch.cuda.synchronize()
        return d_dst.cpu().numpy(), d_st.cpu().numpy()

    out, st = launch(True, descs, src, dst_size)
    assert (st[bad] == 101).all() and (st[valid] == 0).all(), np.unique(st)
    want = np.zeros(dst_size, np.uint8)
    assert (o.seal_batch(descs[valid], keys, kidx, src, want) == 0).all()
    assert np.array_equal(out, want), "sealed bytes differ from the oracle"
    d2 = np.zeros(n, DESC)
    d2["src_off"], d2["dst_off"], d2["len"] = doffs, soffs, sizes + 32
    d2["key_slot"] = descs["key_slot"]
    markers = [] if form == "affine" else [8, 9]
    d2["key_slot"][markers] = [0xFFFFFFFE, 0xFFFFFFFF][: len(markers)]  # invalid / no-session
    ok2 = valid.copy()
    ok2[markers] = False
    wire = out.copy()
    tampered, wrong_idx = [11, 1300], [40]
    for t in tampered:
        wire[int(doffs[t]) + 16 + int(rng.integers(0, int(sizes[t]) + 16))] ^= 0x02
    for t in wrong_idx:
        wire[int(doffs[t]) + 5] ^= 0x80
    back, st2 = launch(False, d2, wire, len(src))
    assert (st2[bad] == 101).all() and (st2[markers] == [13, 14][: len(markers)]).all()
    want2 = np.zeros(len(src), np.uint8)
    wst2 = o.open_batch(d2[ok2], keys, kidx, wire, want2)  # (the oracle takes valid slots only)
    assert (st2[ok2] == wst2).all(), [(i, st2[ok2][i], wst2[i]) for i in np.nonzero(st2[ok2] != wst2)[0][:8]]
    assert (st2[tampered] == 10).all() and (st2[wrong_idx] != 0).all()
    assert np.array_equal(back, want2), "opened bytes differ from the oracle"


def test_randomized_launch_shapes_match_oracle(torch_cuda, gpu, gpu1):
    """Randomized sweep over the launch shapes the host picks kernels from, each
    against the oracle bit for bit: strided batches (random n incl. partial waves,
    P 0..2600, strides and output offsets on and off 128-byte lines -- the wire grid,
    the text grid and the one-wave tail launch -- counters across 2^32), and descriptor
    batches on a 4096-slot and a one-slot context (per-lane, SGPR-key, affine and
    plan-ordered forms) with tampered and wrong-index datagrams.  Bytes outside every
    packet's output must keep their canary value."""
    torch = torch_cuda
    rng = np.random.default_rng(20261017)
    keys = rng.integers(0, 256, (4096, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, 4096, dtype=np.uint64).astype(np.uint32)
    gpu.set_keys(0, keys, kidx)
    gpu1.set_keys(0, keys[:1], kidx[:1])
    for it in range(32):  # strided
        n = int(rng.choice([1, 63, 64, 65, 511, 512, 1000, 2049]))
        P = int(rng.choice([0, 1, 15, 16, 17, 127, 128, 129, 1350, 1366, int(rng.integers(0, 2600))]))
        Ss = synth.round_up(P + int(rng.choice([0, 16, 48, 160])), 16) or 16
        Sw = synth.round_up(P + 32 + int(rng.choice([0, 16, 96, 250])), 16)
        Sp = synth.round_up(P + int(rng.choice([0, 16, 112, 200])), 16) or 16
        po = int(rng.choice([0, 16, 32, 128]))   # open's plaintext offset into its buffer
        wo = int(rng.choice([0, 16, 128]))      # seal's datagram offset
        base = int(rng.choice([0, 2**32 - 40, int(rng.integers(0, 2**62))]))
        slot = int(rng.integers(0, 4096))
        src = rng.integers(0, 256, n * Ss + 16, dtype=np.uint8)
        d_src = to_dev(torch, src)
        wire = torch.full((n * Sw + wo + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        gpu.seal_strided(n, P, slot, base, d_src, Ss, wire.data_ptr() + wo, Sw, st)
        torch.cuda.synchronize()
        assert (st == 0).all(), (it, n, P)
        descs = np.zeros(n, DESC)
        descs["src_off"] = np.arange(n, dtype=np.int64) * Ss
        descs["dst_off"] = wo + np.arange(n, dtype=np.int64) * Sw
        descs["counter"] = (np.uint64(base) + np.arange(n, dtype=np.uint64))
        descs["len"] = P
        descs["key_slot"] = slot
        want = np.full(n * Sw + wo + 64, 0xA5, np.uint8)
        assert (o.seal_batch(descs, keys, kidx, src, want) == 0).all()
        assert np.array_equal(wire.cpu().numpy(), want), f"strided seal {it}: n={n} P={P} Sw={Sw} wo={wo}"
        back = torch.full((n * Sp + po + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        st.fill_(-1)
        gpu.open_strided(n, P + 32, slot, wire.data_ptr() + wo, Sw, back.data_ptr() + po, Sp, st)
        torch.cuda.synchronize()
        assert (st == 0).all(), (it, n, P)
        exp = np.full(n * Sp + po + 64, 0x5A, np.uint8)
        for i in range(n):
            exp[po + i * Sp:po + i * Sp + P] = src[i * Ss:i * Ss + P]
        assert np.array_equal(back.cpu().numpy(), exp), f"strided open {it}: n={n} P={P} Sp={Sp} po={po}"
    for it in range(24):  # descriptor batches
        ctx = gpu1 if it % 3 == 0 else gpu
        nk = 1 if ctx is gpu1 else 4096
        n = int(rng.integers(1, 3000))
        affine = it % 2 == 1
        if affine:
            P = int(rng.choice([0, 64, 1350, 1400]))
            sizes = np.full(n, P, np.int64)
            S = synth.round_up(P + 32 + int(rng.choice([0, 16, 80])), 16)
            soffs = 16 * int(rng.integers(0, 8)) + S * np.arange(n, dtype=np.int64)
            doffs = 16 * int(rng.integers(0, 8)) + S * np.arange(n, dtype=np.int64)
            src = np.zeros(int(soffs[-1]) + S + 64, np.uint8)
            for i, p in enumerate(synth.host_payloads(sizes, seed=it)):
                src[soffs[i]:soffs[i] + P] = np.frombuffer(p, np.uint8)
            dst_size = int(doffs[-1]) + S + 64
        else:
            sizes = rng.choice([0, 1, 16, 64, 200, 576, 1350, 1500, 4000, 8900], n)
            src, soffs = pack(synth.host_payloads(sizes, seed=100 + it))
            soffs = np.array(soffs, np.int64)
            doffs, pos = np.zeros(n, np.int64), 0
            for i in rng.permutation(n):
                doffs[i] = pos
                pos = synth.round_up(pos + int(sizes[i]) + 32 + 16 * int(rng.integers(0, 3)), 16)
            dst_size = pos + 64
        descs = np.zeros(n, DESC)
        descs["src_off"], descs["dst_off"], descs["len"] = soffs, doffs, sizes
        descs["counter"] = rng.integers(0, 2**63, n, dtype=np.uint64)
        descs["key_slot"] = rng.integers(0, nk, n).astype(np.uint32)
        ordered = not affine and it % 4 == 0

        def launch(seal, d, src_b, size, fill):
            d_descs = to_dev(torch, d.view(np.uint8))
            d_src = to_dev(torch, src_b)
            d_dst = torch.full((max(size, 16),), fill, dtype=torch.uint8, device="cuda")
            d_st = torch.full((len(d),), -1, dtype=torch.int32, device="cuda")
            if ordered:
                order = torch.zeros(len(d), dtype=torch.int32, device="cuda")
                scratch = torch.zeros(262144 // 4, dtype=torch.int32, device="cuda")
                ctx.plan_batch(seal, d_descs, len(d), order, scratch)
                (ctx.seal_batch_ordered if seal else ctx.open_batch_ordered)(
                    d_descs, order, len(d), d_src, d_dst, d_st)
            else:
                (ctx.seal_batch if seal else ctx.open_batch)(d_descs, len(d), d_src, d_dst, d_st)
            torch.cuda.synchronize()
            return d_dst.cpu().numpy(), d_st.cpu().numpy()

        out, st = launch(True, descs, src, dst_size, 0xC3)
        want = np.full(max(dst_size, 16), 0xC3, np.uint8)
        assert (o.seal_batch(descs, keys[:nk], kidx[:nk], src, want) == 0).all()
        assert (st == 0).all() and np.array_equal(out, want), f"desc seal {it}: n={n} affine={affine} nk={nk}"
        d2 = np.zeros(n, DESC)
        d2["src_off"], d2["dst_off"], d2["len"], d2["key_slot"] = doffs, soffs, sizes + 32, descs["key_slot"]
        wire = out.copy()
        bad = rng.choice(n, size=min(n, 3), replace=False)
        wire[int(doffs[bad[0]]) + 16 + int(rng.integers(0, int(sizes[bad[0]]) + 16))] ^= 0x08
        if len(bad) > 1:
            wire[int(doffs[bad[1]]) + 4] ^= 0x80   # receiver index
        back, st2 = launch(False, d2, wire, len(src), 0x3C)
        want2 = np.full(max(len(src), 16), 0x3C, np.uint8)
        wst2 = o.open_batch(d2, keys[:nk], kidx[:nk], wire, want2)
        assert (st2 == wst2).all() and (wst2[bad[0]] == 10), f"desc open status {it}"
        assert np.array_equal(back, want2), f"desc open {it}: n={n} affine={affine} nk={nk} ordered={ordered}"


@pytest.mark.parametrize("grid", ["wire_padded", "text"])
def test_full_size_open_failures_in_every_group(torch_cuda, gpu, grid):
    """1M x 1350 B opened with failures spread over the whole batch -- so every
    persistent workgroup meets them in its later groups too (each walks 4 groups at
    this size): flipped ciphertext and tag bytes (InvalidAeadTag, plaintext zeroed),
    wrong receiver index and wrong message type (the packet left untouched).  Wire grid
    with slot padding (the bench's open) and NepTUN's offset-0 open (text grid); every
    other packet back bit for bit, statuses equal to the oracle's on sampled packets."""
    torch = torch_cuda
    n, P, S = 1 << 20, 1350, 1408
    keys = synth.keys(1, seed=31)
    gpu.set_keys(0, keys, np.array([synth.RECEIVER_IDX], np.uint32))
    rng = np.random.default_rng(31)
    pt = synth.device_payloads(n, P, S, "cuda", offset=16)
    wire = torch.zeros(n * S, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.seal_strided(n, P, 0, 5, pt.data_ptr() + 16, S, wire, S, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    picks = rng.choice(n, size=4000, replace=False)
    ct_bad, tag_bad, idx_bad, type_bad = np.array_split(picks, 4)
    w = wire.view(n, S)
    for rows, off in ((ct_bad, rng.integers(16, 16 + P, len(ct_bad))),
                      (tag_bad, rng.integers(16 + P, 32 + P, len(tag_bad)))):
        r_t, c_t = torch.from_numpy(rows).cuda(), torch.from_numpy(off).cuda()
        w[r_t, c_t] ^= 0x20
    w[torch.from_numpy(idx_bad).cuda(), 4] ^= 0x01
    w[torch.from_numpy(type_bad).cuda(), 0] = 2
    back = torch.full((n * S,), 0xCD, dtype=torch.uint8, device="cuda")
    st.fill_(-1)
    o_off = 16 if grid == "wire_padded" else 0
    gpu.set_slot_padding(grid == "wire_padded")
    try:
        gpu.open_strided(n, P + 32, 0, wire, S, back.data_ptr() + o_off, S, st)
        torch.cuda.synchronize()
    finally:
        gpu.set_slot_padding(False)
    s_h = st.cpu().numpy()
    aead = np.concatenate([ct_bad, tag_bad])
    assert (s_h[aead] == 10).all(), np.unique(s_h[aead])          # InvalidAeadTag + 1
    assert (s_h[idx_bad] == 5).all() and (s_h[type_bad] != 0).all()  # WrongIndex + 1
    good = np.ones(n, bool)
    good[picks] = False
    assert (s_h[good] == 0).all()
    b2 = back.view(n, S)
    g_t = torch.from_numpy(np.nonzero(good)[0]).cuda()
    assert torch.equal(b2[g_t, o_off:o_off + P], pt.view(n, S)[g_t, 16:16 + P])
    assert not bool(b2[torch.from_numpy(aead).cuda(), o_off:o_off + P].any()), "failed tags not zeroed"
    nogo = torch.from_numpy(np.concatenate([idx_bad, type_bad])).cuda()
    assert bool((b2[nogo, o_off:o_off + P] == 0xCD).all()), "refused packets written"
    # the oracle agrees on a sample of each kind
    wh = wire.view(n, S)
    for rows in (ct_bad[:8], tag_bad[:8], idx_bad[:8], good.nonzero()[0][:: n // 16]):
        for r in rows:
            code, _ = o.receive_packet_data(keys[0].tobytes(), synth.RECEIVER_IDX,
                                            wh[int(r), :P + 32].cpu().numpy().tobytes())
            assert code == int(s_h[r]), (int(r), code, int(s_h[r]))


@pytest.mark.parametrize("form", ["per_lane", "key1", "ordered"])
def test_descriptor_packets_below_the_fast_anchor(torch_cuda, gpu, gpu1, form):
    """the descriptor kernels' fast addressing anchors each wave at
    its first staged packet - 1 GiB.  A packet of the same wave that starts just below
    that anchor and ends past it (lanes 1 of these waves, 16 .. 1344 bytes below it on
    both the input and the output side) must not take the 32-bit fast path (its offset
    would wrap) -- sealed and opened bit-exact against the oracle, with every byte
    outside the packets left at its canary value, in the per-lane, one-slot (SGPR
    key) and plan-ordered kernel forms."""
    torch = torch_cuda
    ctx = gpu1 if form == "key1" else gpu
    rng = np.random.default_rng(404)
    nk = 1 if ctx is gpu1 else 64
    keys = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, nk, dtype=np.uint64).astype(np.uint32)
    ctx.set_keys(0, keys, kidx)
    P, S, GiB = 1350, 1408, 1 << 30
    H = GiB + (1 << 20)            # lane 0 of every wave lives above 1 GiB
    deltas = [-16, -48, -512, -1344]
    n = 64 * len(deltas)
    offs = np.zeros(n, np.int64)
    for w, dl in enumerate(deltas):
        for lane in range(64):
            offs[64 * w + lane] = H + (64 * w + lane) * S
        offs[64 * w + 1] = offs[64 * w] - GiB + dl   # straddles the wave's anchor
    size = int(offs.max()) + S + 4096
    payloads = synth.host_payloads(np.full(n, P), seed=405)
    src = np.full(size, 0x11, np.uint8)
    for i in range(n):
        src[offs[i]:offs[i] + P] = np.frombuffer(payloads[i], np.uint8)
    descs = np.zeros(n, DESC)
    descs["src_off"], descs["dst_off"], descs["len"] = offs, offs, P
    descs["counter"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    descs["key_slot"] = rng.integers(0, nk, n).astype(np.uint32)

    def launch(seal, d, src_b, fill):
        d_descs = to_dev(torch, d.view(np.uint8))
        d_src = to_dev(torch, src_b)
        d_dst = torch.full((size,), fill, dtype=torch.uint8, device="cuda")
        d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        if form == "ordered":
            order = torch.zeros(n, dtype=torch.int32, device="cuda")
            scratch = torch.zeros(262144 // 4, dtype=torch.int32, device="cuda")
            ctx.plan_batch(seal, d_descs, n, order, scratch)
            (ctx.seal_batch_ordered if seal else ctx.open_batch_ordered)(
                d_descs, order, n, d_src, d_dst, d_st)
        else:
            (ctx.seal_batch if seal else ctx.open_batch)(d_descs, n, d_src, d_dst, d_st)
        torch.cuda.synchronize()
        del d_src
        return d_dst, d_st.cpu().numpy()

    wire_d, st = launch(True, descs, src, 0xC3)
    want = np.full(size, 0xC3, np.uint8)
    assert (o.seal_batch(descs, keys, kidx, src, want) == 0).all()
    assert (st == 0).all(), np.unique(st)
    assert torch.equal(wire_d, to_dev(torch, want)), "sealed bytes (or canaries) differ from the oracle"
    d2 = descs.copy()
    d2["len"] = P + 32
    wire = wire_d.cpu().numpy()
    del wire_d
    back_d, st2 = launch(False, d2, wire, 0x3C)
    want2 = np.full(size, 0x3C, np.uint8)
    assert (o.open_batch(d2, keys, kidx, wire, want2) == 0).all()
    assert (st2 == 0).all(), np.unique(st2)
    assert torch.equal(back_d, to_dev(torch, want2)), "opened bytes (or canaries) differ from the oracle"
