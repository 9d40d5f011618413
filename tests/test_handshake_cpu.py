"""Handshake-side primitives on the CPU (no GPU needed):
  * the oracle (oracle/handshake_model.py) against RFC 7748's vectors, OpenSSL's
    X25519 and the reference's own INITIAL_CHAIN_KEY / INITIAL_CHAIN_HASH
    constants (neptun/src/noise/handshake.rs:29-39, BLAKE2s outputs);
  * the product headers wg_x25519.h / wg_blake2s.h (the device code, compiled
    for the host with g++) against the oracle on random and edge-case inputs.
"""
import hashlib
import json
import os
import random
import subprocess

import pytest

from oracle import handshake_model as H
from oracle import pyoracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "handshake.json")))
CSRC = os.path.join(ROOT, "neptun_amd", "csrc")


def test_oracle_rfc7748_vectors():
    for v in GOLDEN["scalarmult"]:
        assert H.x25519(bytes.fromhex(v["scalar"]), bytes.fromhex(v["u"])).hex() == v["out"]
    k = u = (9).to_bytes(32, "little")
    assert H.x25519(k, u).hex() == GOLDEN["iterated_1"]
    d = GOLDEN["dh"]
    a, b = bytes.fromhex(d["alice_private"]), bytes.fromhex(d["bob_private"])
    assert H.public_key(a).hex() == d["alice_public"]
    assert H.public_key(b).hex() == d["bob_public"]
    assert H.x25519(a, H.public_key(b)).hex() == d["shared"]
    assert H.x25519(b, H.public_key(a)).hex() == d["shared"]


def test_oracle_matches_reference_chain_constants():
    c = GOLDEN["reference_chain_constants"]
    assert list(H.INITIAL_CHAIN_KEY) == c["INITIAL_CHAIN_KEY"]
    assert list(H.INITIAL_CHAIN_HASH) == c["INITIAL_CHAIN_HASH"]


def test_oracle_x25519_matches_openssl():
    o.build()
    rng = random.Random(3)
    for _ in range(300):
        k, u = rng.randbytes(32), rng.randbytes(32)
        ref = o.openssl_x25519(k, u)
        if ref is not None:
            assert H.x25519(k, u) == ref


@pytest.fixture(scope="module")
def harnesses(tmp_path_factory):
    d = tmp_path_factory.mktemp("hs")
    out = {}
    for name in ("x25519", "blake2s"):
        exe = str(d / name)
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", CSRC,
                        os.path.join(ROOT, "tests", "native", f"{name}_harness.cpp"), "-o", exe],
                       check=True)
        out[name] = exe
    return out


def run(exe, lines):
    r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                       check=True, timeout=300)
    return r.stdout.split()


def test_device_x25519_code_matches_oracle_on_host(harnesses):
    rng = random.Random(5)
    p = H.P25519
    points = [0, 1, p - 1, p, p + 1, 2**255 - 1, 2**256 - 1, 9,
              # a point of order 8 and its twist-side neighbours (small-order inputs)
              325606250916557431795983626356110631294008115727848805560023387167927233504]
    cases = [(rng.randbytes(32), (x % 2**256).to_bytes(32, "little")) for x in points]
    cases += [(rng.randbytes(32), rng.randbytes(32)) for _ in range(600)]
    v = GOLDEN["scalarmult"][0]
    cases.append((bytes.fromhex(v["scalar"]), bytes.fromhex(v["u"])))
    out = run(harnesses["x25519"], [k.hex() + " " + u.hex() for k, u in cases])
    assert out == [H.x25519(k, u).hex() for k, u in cases]


def test_device_blake2s_code_matches_hashlib_on_host(harnesses):
    rng = random.Random(7)
    lines, want = [], []
    for _ in range(200):
        k = rng.randbytes(32)
        n = rng.choice([0, 1, 31, 32, 33, 63, 64])
        d = rng.randbytes(n)
        if n == 32:
            lines.append(f"hash {k.hex()} {d.hex()}")
            want.append(H.b2s_hash(k, d).hex())
        else:
            lines.append(f"hash {k.hex()} {d.hex() or '-'}")
            want.append(hashlib.blake2s(d).hexdigest())
        lines.append(f"hmac {k.hex()} {d.hex() or '-'}")
        want.append(H.b2s_hmac(k, d).hex())
        m = rng.randbytes(116)
        lines.append(f"mac {k.hex()} {m.hex()}")
        want.append(H.b2s_keyed_mac_16(k, m).hex())
    assert run(harnesses["blake2s"], lines) == want


def test_model_handshake_round_trip():
    """format_handshake_initiation -> parse_handshake_anon in the model recovers the
    initiator's static key; a flipped bit fails mac1 or the AEAD tag."""
    rng = random.Random(9)
    resp_priv, init_priv = rng.randbytes(32), rng.randbytes(32)
    msg = H.format_handshake_initiation(init_priv, H.public_key(resp_priv), rng.randbytes(32),
                                        77, rng.randbytes(12))
    st, idx, pub = H.parse_handshake_anon(resp_priv, H.public_key(resp_priv), msg)
    assert (st, idx, pub) == (0, 77, H.public_key(init_priv))
    bad = bytearray(msg)
    bad[50] ^= 1
    assert H.parse_handshake_anon(resp_priv, H.public_key(resp_priv), bytes(bad))[0] == H.INVALID_MAC
    assert H.parse_handshake_anon(resp_priv, H.public_key(resp_priv), bytes(bad),
                                  check_mac1=False)[0] == H.INVALID_AEAD_TAG


def test_oracle_xchacha_matches_golden_vectors():
    """Cookie AEAD restatement (HChaCha20 + RFC 8439) vs libsodium's vectors and the
    draft's HChaCha20 KAT (tests/golden/xchacha.json, oracle/gen_golden_xchacha.py)."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "xchacha.json")))
    d = g["hchacha20_draft"]
    assert H.hchacha20(bytes.fromhex(d["key"]), bytes.fromhex(d["nonce"])).hex() == d["subkey"]
    for v in g["vectors"]:
        key, nonce = bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"])
        aad, pt = bytes.fromhex(v["aad"]), bytes.fromhex(v["pt"])
        assert H.hchacha20(key, nonce[:16]).hex() == v["hchacha20_subkey"]
        assert H.xchacha20poly1305_seal(key, nonce, aad, pt).hex() == v["ct_tag"]
        assert H.xchacha20poly1305_open(key, nonce, aad, bytes.fromhex(v["ct_tag"])) == pt


def test_oracle_responder_round_trip_with_initiator():
    """The responder restatement (consume_initiation + format_response,
    handshake.rs:527-613, 853-949) against the initiator side (initiation /
    receive_response, :769-830, 615-695): the initiator accepts the response and
    both ends derive the same session keys (sending of one = receiving of the other)."""
    rng = random.Random(23)
    for psk in (None, rng.randbytes(32)):
        for cookie in (None, rng.randbytes(16)):
            si, sr, ei, er = (rng.randbytes(32) for _ in range(4))
            pi, pr = H.public_key(si), H.public_key(sr)
            ts = rng.randbytes(12)
            msg, ck_i, h_i = H.initiation(si, pr, ei, rng.getrandbits(32), ts)
            st, pidx, t, ck, h, peph = H.consume_initiation(sr, pi, H.x25519(sr, pi), msg)
            assert st == 0 and t == ts
            resp, rk, sk, mac1 = H.format_response(ck, h, peph, pidx, 77, er, pi, psk, cookie)
            assert H.b2s_keyed_mac_16(H.b2s_hash(H.LABEL_MAC1, pi), resp[:60]) == resp[60:76] == mac1
            assert (cookie is None) == (resp[76:] == bytes(16))
            st2, send_i, recv_i = H.receive_response(ck_i, h_i, ei, si, resp, psk)
            assert st2 == 0 and send_i == rk and recv_i == sk
    # the wrong peer key / a damaged timestamp are refused
    st = H.consume_initiation(sr, H.public_key(rng.randbytes(32)), H.x25519(sr, pi), msg)[0]
    assert st == H.WRONG_KEY
    bad = bytearray(msg)
    bad[95] ^= 1
    assert H.consume_initiation(sr, pi, H.x25519(sr, pi), bytes(bad))[0] == H.INVALID_AEAD_TAG
