#!/usr/bin/env python3
"""Generate and cross-check the golden fixtures under tests/golden/.

TEST INFRASTRUCTURE ONLY.  Run in the build container (needs gcc + libcrypto +
node); the GPU box only reads the committed JSON.

Pinning chain (DESIGN.md "Oracle"):
  1. the reference's own KAT, neptun/src/noise/handshake.rs:957-992 (RFC 8439
     2.8.2, run through ring) -- the oracle and OpenSSL must both reproduce it;
  2. RFC 8439 2.5.2 (Poly1305) -- published vector;
  3. NepTUN framing (session.rs:205-302: header 4|idx|LE64 ctr, nonce
     0^4|LE64 ctr, empty AAD, no padding, 16 B tag) applied over three
     independent RFC 8439 implementations -- this oracle (C), OpenSSL 3 EVP,
     node 12 crypto -- which must agree byte for byte on every vector.
The reference has no fixed-key data-packet vectors (all its data-path tests use
OsRng keys, noise/mod.rs:1090-1140), so (3) is the framing's pin.

Usage: python oracle/gen_golden.py [--check-only]
"""
from __future__ import annotations

import json
import os
import random
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pyoracle as o  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
SEED = 0x4E455054554E  # "NEPTUN"


def splitmix_bytes(seed: int, n: int) -> bytes:
    out = bytearray()
    s = seed & 0xFFFFFFFFFFFFFFFF
    while len(out) < n:
        s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


def ossl_frame(key: bytes, idx: int, ctr: int, payload: bytes) -> bytes:
    import ctypes
    out = ctypes.create_string_buffer(len(payload) + 32)
    rc = o.openssl().ossl_format_packet_data(key, idx, ctr, payload, len(payload), out)
    assert rc == 0
    return out.raw


def node_frame(vectors: list[dict]) -> list[str]:
    """Seal the same vectors with node's crypto (third independent implementation)."""
    script = r"""
const crypto = require('crypto');
const vs = JSON.parse(require('fs').readFileSync(0, 'utf8'));
const out = vs.map(v => {
  const key = Buffer.from(v.key, 'hex');
  const nonce = Buffer.alloc(12);
  nonce.writeBigUInt64LE(BigInt(v.counter), 4);
  const c = crypto.createCipheriv('chacha20-poly1305', key, nonce, {authTagLength: 16});
  const ct = Buffer.concat([c.update(Buffer.from(v.payload, 'hex')), c.final()]);
  const hdr = Buffer.alloc(16);
  hdr.writeUInt32LE(4, 0); hdr.writeUInt32LE(v.sending_index, 4);
  hdr.writeBigUInt64LE(BigInt(v.counter), 8);
  return Buffer.concat([hdr, ct, c.getAuthTag()]).toString('hex');
});
process.stdout.write(JSON.stringify(out));
"""
    # counters travel as decimal strings: JSON numbers lose bits above 2^53 in JS
    payload = [dict(v, counter=str(v["counter"])) for v in vectors]
    res = subprocess.run(["node", "-e", script], input=json.dumps(payload).encode(),
                         capture_output=True)
    if res.returncode:
        raise RuntimeError(res.stderr.decode())
    return json.loads(res.stdout)


def kat() -> dict:
    # neptun/src/noise/handshake.rs:957-992 (RFC 8439 2.8.2)
    pt = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip "
          b"for the future, sunscreen would be it.")
    key = bytes(range(0x80, 0xA0))
    nonce = bytes([0x07, 0, 0, 0]) + bytes(range(0x40, 0x48))
    aad = bytes.fromhex("50515253c0c1c2c3c4c5c6c7")
    ct_exp = bytes.fromhex(
        "d31a8d34648e60db7b86afbc53ef7ec2a4aded51296e08fea9e2b5a736ee62d63dbea45e8ca967128"
        "2fafb69da92728b1a71de0a9e060b2905d6a5b67ecd3b3692ddbd7f2d778b8c9803aee328091b58fa"
        "b324e4fad675945585808b4831d7bc3ff4def08e4b7a9de576d26586cec64b6116")
    tag_exp = bytes.fromhex("1ae10b594f09e26a7e902ecbd0600691")
    ct, tag = o.aead_seal(key, nonce, aad, pt)
    assert (ct, tag) == (ct_exp, tag_exp), "oracle fails the reference KAT"
    import ctypes
    c2 = ctypes.create_string_buffer(len(pt))
    t2 = ctypes.create_string_buffer(16)
    o.openssl().ossl_aead_seal(key, nonce, aad, len(aad), pt, len(pt), c2, t2)
    assert (c2.raw, t2.raw) == (ct_exp, tag_exp), "OpenSSL fails the reference KAT"
    # RFC 8439 2.5.2 Poly1305
    pk = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    ptag = o.poly1305(pk, b"Cryptographic Forum Research Group")
    assert ptag.hex() == "a8061dc1305136c6c22b8baf0c0127a9"
    return {
        "source": "neptun/src/noise/handshake.rs:957-992 (RFC 8439 2.8.2 via ring)",
        "aead": [{"key": key.hex(), "nonce": nonce.hex(), "aad": aad.hex(), "pt": pt.hex(),
                  "ct": ct_exp.hex(), "tag": tag_exp.hex()}],
        "poly1305": [{"source": "RFC 8439 2.5.2", "key": pk.hex(),
                      "msg": b"Cryptographic Forum Research Group".hex(),
                      "tag": "a8061dc1305136c6c22b8baf0c0127a9"}],
    }


SIZES = [0, 1, 2, 15, 16, 17, 31, 32, 33, 48, 63, 64, 65, 100, 127, 128, 129, 191, 192, 255,
         256, 576, 1024, 1350, 1400, 1420, 1500, 2048, 8192, 8900]
COUNTERS = [0, 1, 2, 255, 0xFFFFFFFF, 0x100000000, 0x123456789ABCDEF0, (1 << 63),
            0xFFFFFFFFFFFFFFFE, 0xFFFFFFFFFFFFFFFF]


def data_vectors() -> list[dict]:
    rng = random.Random(SEED)
    keys = [splitmix_bytes(SEED + 1 + k, 32) for k in range(3)]
    vecs = []
    for i, size in enumerate(SIZES):
        key = keys[i % 3]
        ctr = COUNTERS[i % len(COUNTERS)]
        idx = rng.getrandbits(32)
        payload = splitmix_bytes(SEED ^ (i * 7919), size)
        wire = o.format_packet_data(key, idx, ctr, payload)
        vecs.append({"key": key.hex(), "sending_index": idx, "counter": ctr,
                     "payload": payload.hex(), "wire": wire.hex()})
    # every counter edge at the headline size
    for j, ctr in enumerate(COUNTERS):
        key = keys[j % 3]
        payload = splitmix_bytes(SEED + 1000 + j, 1350)
        wire = o.format_packet_data(key, 0x00ABCD01, ctr, payload)
        vecs.append({"key": key.hex(), "sending_index": 0x00ABCD01, "counter": ctr,
                     "payload": payload.hex(), "wire": wire.hex()})
    return vecs


def tamper_vectors(vecs: list[dict]) -> list[dict]:
    """Datagrams that must fail with InvalidAeadTag (session.rs:290-296)."""
    out = []
    for k, v in enumerate(vecs[:: max(1, len(vecs) // 8)]):
        wire = bytearray(bytes.fromhex(v["wire"]))
        p = len(wire) - 32
        cases = [("tag_bit", 16 + p + (k % 16))]
        if p:
            cases.append(("ct_bit", 16 + (k * 37) % p))
        cases.append(("counter_bit", 8 + k % 8))
        for name, pos in cases:
            w = bytearray(wire)
            w[pos] ^= 1 << (k % 8)
            out.append({"key": v["key"], "receiving_index": v["sending_index"], "case": name,
                        "wire": bytes(w).hex(), "status": 10})
    # wrong key
    v = vecs[23]
    out.append({"key": "00" * 32, "receiving_index": v["sending_index"], "case": "wrong_key",
                "wire": v["wire"], "status": 10})
    return out


def cross_check(n_random: int = 3000) -> int:
    """Oracle vs OpenSSL on random keys/counters/sizes 0..9000 (incl. counters >= 2^32)."""
    rng = random.Random(SEED + 7)
    for t in range(n_random):
        size = rng.choice([rng.randrange(0, 64), rng.randrange(0, 9001), 1350])
        key = rng.randbytes(32)
        ctr = rng.choice([rng.getrandbits(64), rng.getrandbits(32), rng.randrange(0, 4096)])
        idx = rng.getrandbits(32)
        payload = rng.randbytes(size)
        a = o.format_packet_data(key, idx, ctr, payload)
        b = ossl_frame(key, idx, ctr, payload)
        assert a == b, f"oracle != OpenSSL at size={size} ctr={ctr}"
        st, pt = o.receive_packet_data(key, idx, a)
        assert st == 0 and pt == payload
    return n_random


def main() -> None:
    check_only = "--check-only" in sys.argv
    o.build()
    k = kat()
    n = cross_check()
    vecs = data_vectors()
    node = node_frame(vecs)
    for v, w in zip(vecs, node):
        assert v["wire"] == w, "oracle != node crypto"
        assert ossl_frame(bytes.fromhex(v["key"]), v["sending_index"], v["counter"],
                          bytes.fromhex(v["payload"])).hex() == v["wire"]
    tam = tamper_vectors(vecs)
    for t in tam:
        st, _ = o.receive_packet_data(bytes.fromhex(t["key"]), t["receiving_index"],
                                      bytes.fromhex(t["wire"]))
        assert st == 10, t["case"]
    print(f"KAT ok; {n} random oracle==OpenSSL; {len(vecs)} framed vectors oracle==OpenSSL==node; "
          f"{len(tam)} tamper cases reject")
    if check_only:
        return
    os.makedirs(GOLDEN, exist_ok=True)
    meta = {"generator": "oracle/gen_golden.py", "framing": "neptun/src/noise/session.rs:205-302",
            "implementations_agreeing": ["oracle/neptun_oracle.c", "OpenSSL 3 EVP_chacha20_poly1305",
                                         "node v12 crypto chacha20-poly1305"]}
    with open(os.path.join(GOLDEN, "rfc8439_kat.json"), "w") as f:
        json.dump(k, f, indent=1)
    with open(os.path.join(GOLDEN, "data_packets.json"), "w") as f:
        json.dump({"meta": meta, "vectors": vecs}, f, indent=0)
    with open(os.path.join(GOLDEN, "tamper.json"), "w") as f:
        json.dump({"meta": meta, "expected_status": "10 = WireGuardError::InvalidAeadTag + 1",
                   "vectors": tam}, f, indent=0)


if __name__ == "__main__":
    main()
