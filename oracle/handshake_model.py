"""Handshake-side primitives of NepTUN, restated in Python -- TEST INFRASTRUCTURE ONLY.

The checker for the GPU handshake kernels (neptun_amd/csrc/wg_handshake.hip):
  X25519                      RFC 7748 section 5 (x25519-dalek in the reference,
                              neptun/src/lib.rs:21-24; not vendored)
  b2s_hash / b2s_hmac / b2s_hmac2 / b2s_keyed_mac_16
                              neptun/src/noise/handshake.rs:42-91 (BLAKE2s = RFC 7693,
                              HMAC = RFC 2104 over BLAKE2s, 64-byte block)
  parse_handshake_anon        handshake.rs:367-412
  mac1 check                  rate_limiter.rs:172-195 (mac1_key = HASH(LABEL_MAC1 || pub))
  format_handshake_initiation handshake.rs:769-830 + append_mac1_and_mac2 :732-765
                              (initiator side, used to build test messages; the
                              ephemeral key and timestamp come from the caller)
Pinned by RFC 7748's test vectors, OpenSSL's X25519 (oracle/openssl_ref.c) and the
reference's own INITIAL_CHAIN_KEY / INITIAL_CHAIN_HASH constants (handshake.rs:29-39),
which are BLAKE2s outputs (tests/test_handshake_cpu.py).
"""
from __future__ import annotations

import hashlib
import hmac as _hmac

from oracle import pyoracle as o

P25519 = 2**255 - 19
A24 = 121665
LABEL_MAC1 = b"mac1----"
LABEL_COOKIE = b"cookie--"
CONSTRUCTION = b"Noise_IKpsk2_25519_ChaChaPoly_BLAKE2s"
IDENTIFIER = b"WireGuard v1 zx2c4 Jason@zx2c4.com"
HANDSHAKE_INIT, HANDSHAKE_INIT_SZ = 1, 148
INVALID_MAC, INVALID_AEAD_TAG, WRONG_PACKET_TYPE = 9, 10, 4  # WireGuardError index + 1


def clamp(k: bytes) -> int:
    b = bytearray(k)
    b[0] &= 248
    b[31] &= 127
    b[31] |= 64
    return int.from_bytes(b, "little")


def x25519(k: bytes, u: bytes) -> bytes:
    """RFC 7748 5: Montgomery ladder on curve25519 (constant structure, Python ints)."""
    kk = clamp(k)
    x1 = int.from_bytes(u, "little") & ((1 << 255) - 1)
    x2, z2, x3, z3, swap = 1, 0, x1, 1, 0
    for t in range(254, -1, -1):
        kt = (kk >> t) & 1
        swap ^= kt
        if swap:
            x2, x3, z2, z3 = x3, x2, z3, z2
        swap = kt
        a = (x2 + z2) % P25519
        aa = a * a % P25519
        b = (x2 - z2) % P25519
        bb = b * b % P25519
        e = (aa - bb) % P25519
        c = (x3 + z3) % P25519
        d = (x3 - z3) % P25519
        da = d * a % P25519
        cb = c * b % P25519
        x3 = (da + cb) ** 2 % P25519
        z3 = x1 * (da - cb) ** 2 % P25519
        x2 = aa * bb % P25519
        z2 = e * (aa + A24 * e) % P25519
    if swap:
        x2, x3, z2, z3 = x3, x2, z3, z2
    return (x2 * pow(z2, P25519 - 2, P25519) % P25519).to_bytes(32, "little")


def public_key(k: bytes) -> bytes:
    return x25519(k, (9).to_bytes(32, "little"))


def b2s_hash(d1: bytes, d2: bytes = b"") -> bytes:
    return hashlib.blake2s(d1 + d2).digest()


def b2s_hmac(key: bytes, d1: bytes, d2: bytes = b"") -> bytes:
    return _hmac.new(key, d1 + d2, hashlib.blake2s).digest()


def b2s_keyed_mac_16(key: bytes, d1: bytes) -> bytes:
    return hashlib.blake2s(d1, key=key, digest_size=16).digest()


INITIAL_CHAIN_KEY = b2s_hash(CONSTRUCTION)
INITIAL_CHAIN_HASH = b2s_hash(INITIAL_CHAIN_KEY, IDENTIFIER)


def _nonce0() -> bytes:
    return bytes(12)  # counter 0 (handshake.rs:101-117)


def format_handshake_initiation(static_private: bytes, peer_static_public: bytes,
                                ephemeral_private: bytes, sender_index: int, timestamp: bytes,
                                cookie: bytes | None = None) -> bytes:
    """handshake.rs:769-830 with the random ephemeral key and TAI64N stamp supplied."""
    static_public = public_key(static_private)
    ck = INITIAL_CHAIN_KEY
    h = b2s_hash(INITIAL_CHAIN_HASH, peer_static_public)
    eph_pub = public_key(ephemeral_private)
    h = b2s_hash(h, eph_pub)
    ck = b2s_hmac(b2s_hmac(ck, eph_pub), b"\x01")
    temp = b2s_hmac(ck, x25519(ephemeral_private, peer_static_public))
    ck = b2s_hmac(temp, b"\x01")
    key = b2s_hmac(temp, ck, b"\x02")
    ct, tag = o.aead_seal(key, _nonce0(), h, static_public)
    enc_static = ct + tag
    h = b2s_hash(h, enc_static)
    temp = b2s_hmac(ck, x25519(static_private, peer_static_public))
    ck = b2s_hmac(temp, b"\x01")
    key = b2s_hmac(temp, ck, b"\x02")
    ct, tag = o.aead_seal(key, _nonce0(), h, timestamp)
    enc_ts = ct + tag
    msg = (HANDSHAKE_INIT.to_bytes(4, "little") + sender_index.to_bytes(4, "little") + eph_pub +
           enc_static + enc_ts)
    mac1 = b2s_keyed_mac_16(b2s_hash(LABEL_MAC1, peer_static_public), msg)
    mac2 = b2s_keyed_mac_16(cookie, msg + mac1) if cookie else bytes(16)
    return msg + mac1 + mac2


def parse_handshake_anon(static_private: bytes, static_public: bytes, msg: bytes,
                         check_mac1: bool = True) -> tuple[int, int, bytes]:
    """-> (status, peer_index, peer_static_public); status 0 = Ok.

    mac1 first (rate_limiter.rs:187-195), then handshake.rs:367-412."""
    if len(msg) != HANDSHAKE_INIT_SZ or int.from_bytes(msg[:4], "little") != HANDSHAKE_INIT:
        return WRONG_PACKET_TYPE, 0, bytes(32)
    if check_mac1:
        want = b2s_keyed_mac_16(b2s_hash(LABEL_MAC1, static_public), msg[:-32])
        if want != msg[-32:-16]:
            return INVALID_MAC, 0, bytes(32)
    peer_index = int.from_bytes(msg[4:8], "little")
    eph = msg[8:40]
    h = b2s_hash(b2s_hash(INITIAL_CHAIN_HASH, static_public), eph)
    ck = b2s_hmac(b2s_hmac(INITIAL_CHAIN_KEY, eph), b"\x01")
    temp = b2s_hmac(ck, x25519(static_private, eph))
    ck = b2s_hmac(temp, b"\x01")
    key = b2s_hmac(temp, ck, b"\x02")
    pt = o.aead_open(key, _nonce0(), h, msg[40:72], msg[72:88])
    if pt is None:
        return INVALID_AEAD_TAG, peer_index, bytes(32)
    return 0, peer_index, pt
