"""The CPU oracle against the committed golden vectors (tests/golden/).

Pins: the reference's own KAT (neptun/src/noise/handshake.rs:957-992), RFC 8439
2.5.2, and NepTUN-framed packets (session.rs:205-302) on which three
independent RFC 8439 implementations agree (oracle/gen_golden.py).
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as o

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_reference_kat_seal_open():
    k = load("rfc8439_kat.json")
    for v in k["aead"]:
        key, nonce, aad = (bytes.fromhex(v[x]) for x in ("key", "nonce", "aad"))
        pt = bytes.fromhex(v["pt"])
        ct, tag = o.aead_seal(key, nonce, aad, pt)
        assert ct.hex() == v["ct"] and tag.hex() == v["tag"]
        assert o.aead_open(key, nonce, aad, ct, tag) == pt


def test_reference_kat_tampered_tag_rejected():
    v = load("rfc8439_kat.json")["aead"][0]
    key, nonce, aad = (bytes.fromhex(v[x]) for x in ("key", "nonce", "aad"))
    tag = bytearray(bytes.fromhex(v["tag"]))
    tag[0] ^= 1
    assert o.aead_open(key, nonce, aad, bytes.fromhex(v["ct"]), bytes(tag)) is None


def test_poly1305_vector():
    for v in load("rfc8439_kat.json")["poly1305"]:
        assert o.poly1305(bytes.fromhex(v["key"]), bytes.fromhex(v["msg"])).hex() == v["tag"]


def test_rfc8439_chacha20_block_vector():
    # RFC 8439 2.3.2
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a00000000")
    out = o.chacha20_block(key, 1, nonce)
    assert out[:16].hex() == "10f1e7e4d13b5915500fdd1fa32071c4"
    assert out[-16:].hex() == "b5129cd1de164eb9cbd083e8a2503c4e"


@pytest.mark.parametrize("v", load("data_packets.json")["vectors"],
                         ids=lambda v: f"len{len(v['payload']) // 2}-ctr{v['counter']:x}")
def test_framed_packets(v):
    key = bytes.fromhex(v["key"])
    payload = bytes.fromhex(v["payload"])
    wire = o.format_packet_data(key, v["sending_index"], v["counter"], payload)
    assert wire.hex() == v["wire"]
    # header: LE32 4 | LE32 idx | LE64 counter (session.rs:221-227), length P + 32
    assert wire[:4] == (4).to_bytes(4, "little")
    assert wire[4:8] == v["sending_index"].to_bytes(4, "little")
    assert wire[8:16] == v["counter"].to_bytes(8, "little")
    assert len(wire) == len(payload) + 32
    st, pt = o.receive_packet_data(key, v["sending_index"], wire)
    assert st == 0 and pt == payload


def test_tampered_datagrams_rejected():
    for v in load("tamper.json")["vectors"]:
        st, _ = o.receive_packet_data(bytes.fromhex(v["key"]), v["receiving_index"],
                                      bytes.fromhex(v["wire"]))
        assert st == v["status"] == 10, v["case"]


def test_header_errors():
    v = load("data_packets.json")["vectors"][5]
    key, wire = bytes.fromhex(v["key"]), bytes.fromhex(v["wire"])
    assert o.receive_packet_data(key, v["sending_index"] ^ 1, wire)[0] == 5   # WrongIndex
    assert o.receive_packet_data(key, v["sending_index"], wire[:31])[0] == 13  # InvalidPacket
    bad = bytearray(wire)
    bad[0] = 1
    assert o.receive_packet_data(key, v["sending_index"], bytes(bad))[0] == 13


def test_batch_forms_match_single():
    rng = np.random.default_rng(3)
    n = 40
    sizes = rng.integers(0, 3000, n)
    keys = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    kidx = rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
    src = np.zeros(int(sizes.sum()) + 64 * n, np.uint8)
    dst = np.zeros(int(sizes.sum()) + 64 * n, np.uint8)
    descs = np.zeros(n, o.DESC_DTYPE)
    so = do = 0
    for i, s in enumerate(sizes):
        src[so:so + s] = rng.integers(0, 256, s, dtype=np.uint8)
        descs[i] = (so, do, rng.integers(0, 2**63), s, i % 4)
        so += int(s) + 16
        do += int(s) + 48
    st = o.seal_batch(descs, keys, kidx, src, dst)
    assert (st == 0).all()
    for i in range(n):
        d = descs[i]
        want = o.format_packet_data(keys[d["key_slot"]].tobytes(), int(kidx[d["key_slot"]]),
                                    int(d["counter"]), src[d["src_off"]:d["src_off"] + d["len"]].tobytes())
        assert dst[d["dst_off"]:d["dst_off"] + d["len"] + 32].tobytes() == want


def test_chunked_whole_batch_check_finds_every_corruption():
    """tests/oracle_chunks.py (the GPU suite's whole-batch oracle comparison) run on
    host tensors: a correct batch passes in full, and a flipped byte in any packet --
    including one in a chunk's last packet -- is reported by index."""
    import torch
    from oracle_chunks import chunk_bounds, seal_matches_oracle
    from tools import synth
    rng = np.random.default_rng(8)
    sizes = rng.choice([0, 1, 64, 1350, 8900], 3000).astype(np.int64)
    slot = (sizes + 32 + 127) // 128 * 128
    starts = np.zeros(len(sizes), np.int64)
    starts[1:] = np.cumsum(slot)[:-1]
    end = int(slot.sum())
    src = rng.integers(0, 256, end, dtype=np.uint8)
    d = np.zeros(len(sizes), o.DESC_DTYPE)
    d["src_off"], d["dst_off"], d["len"] = starts + 16, starts, sizes
    d["counter"] = rng.integers(0, 2**63, len(sizes), dtype=np.uint64)
    d["key_slot"] = rng.integers(0, 4, len(sizes))
    keys = synth.keys(4, seed=3)
    kidx = np.arange(4, dtype=np.uint32) + 9
    wire = np.zeros(end, np.uint8)
    assert (o.seal_batch(d, keys, kidx, src, wire) == 0).all()
    bounds = chunk_bounds(starts, end, 1 << 16)
    assert bounds[0][0] == 0 and bounds[-1][1] == len(sizes)
    assert all(a[1] == b[0] for a, b in zip(bounds, bounds[1:]))
    t_src, t_wire = torch.from_numpy(src), torch.from_numpy(wire.copy())
    r = seal_matches_oracle(t_src, t_wire, d, starts, end, keys, kidx, chunk_bytes=1 << 16)
    assert r == {"checked": 3000, "payload_bytes": int(sizes.sum()), "mismatches": 0, "bad": []}
    last = bounds[1][1] - 1
    for i in (5, last):
        t_wire[int(starts[i]) + 4] ^= 1   # the receiver index
    r = seal_matches_oracle(t_src, t_wire, d, starts, end, keys, kidx, chunk_bytes=1 << 16)
    assert r["mismatches"] == 2 and r["bad"] == [5, last]


def test_chunked_check_fails_when_the_oracle_writes_nothing(monkeypatch):
    """The whole-batch check must not pass vacuously: an oracle that reports status 0
    but writes no byte (or only part of a packet) leaves the sentinel behind, and every
    packet it skipped is reported (the expected buffer used to start as
    the GPU's own output)."""
    import torch
    import oracle_chunks
    from tools import synth
    rng = np.random.default_rng(9)
    sizes = rng.choice([0, 5, 64, 1350], 400).astype(np.int64)
    slot = (sizes + 32 + 127) // 128 * 128
    starts = np.zeros(len(sizes), np.int64)
    starts[1:] = np.cumsum(slot)[:-1]
    end = int(slot.sum())
    src = rng.integers(0, 256, end, dtype=np.uint8)
    d = np.zeros(len(sizes), o.DESC_DTYPE)
    d["src_off"], d["dst_off"], d["len"] = starts + 16, starts, sizes
    keys = synth.keys(1, seed=4)
    kidx = np.array([7], np.uint32)
    wire = np.zeros(end, np.uint8)
    assert (o.seal_batch(d, keys, kidx, src, wire) == 0).all()
    t_src, t_wire = torch.from_numpy(src), torch.from_numpy(wire)
    real = o.seal_batch

    def lazy(descs, *a):  # status 0 for all, bytes for none
        return np.zeros(len(descs), np.int32)

    def partial(descs, k, ki, s, dst):  # every packet but its last byte
        st = real(descs, k, ki, s, dst)
        for j in range(len(descs)):
            dst[int(descs["dst_off"][j]) + int(descs["len"][j]) + 31] ^= 0xFF
        return st

    monkeypatch.setattr(oracle_chunks.o, "seal_batch", lazy)
    r = oracle_chunks.seal_matches_oracle(t_src, t_wire, d, starts, end, keys, kidx, chunk_bytes=1 << 15)
    assert r["mismatches"] == len(sizes)
    monkeypatch.setattr(oracle_chunks.o, "seal_batch", partial)
    r = oracle_chunks.seal_matches_oracle(t_src, t_wire, d, starts, end, keys, kidx, chunk_bytes=1 << 15)
    assert r["mismatches"] == len(sizes)
    monkeypatch.setattr(oracle_chunks.o, "seal_batch", real)
    r = oracle_chunks.seal_matches_oracle(t_src, t_wire, d, starts, end, keys, kidx, chunk_bytes=1 << 15)
    assert r["mismatches"] == 0 and r["checked"] == len(sizes)
