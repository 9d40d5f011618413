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
                              (initiator side: builds test messages and checks the
                              device initiator; the ephemeral key and timestamp
                              come from the caller)
  receive_response            handshake.rs:615-695 (checks the device initiator)
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


def initiation(static_private: bytes, peer_static_public: bytes, ephemeral_private: bytes,
               sender_index: int, timestamp: bytes, cookie: bytes | None = None,
               preshared_key: bytes | None = None):
    """handshake.rs:769-830 with the random ephemeral key and TAI64N stamp supplied.
    -> (message, chaining_key, hash): the InitSent state receive_response needs."""
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
    h = b2s_hash(h, enc_ts)
    msg = (HANDSHAKE_INIT.to_bytes(4, "little") + sender_index.to_bytes(4, "little") + eph_pub +
           enc_static + enc_ts)
    mac1 = b2s_keyed_mac_16(b2s_hash(LABEL_MAC1, peer_static_public), msg)
    mac2 = b2s_keyed_mac_16(cookie, msg + mac1) if cookie else bytes(16)
    return msg + mac1 + mac2, ck, h


def format_handshake_initiation(static_private: bytes, peer_static_public: bytes,
                                ephemeral_private: bytes, sender_index: int, timestamp: bytes,
                                cookie: bytes | None = None) -> bytes:
    return initiation(static_private, peer_static_public, ephemeral_private, sender_index,
                      timestamp, cookie)[0]


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


# ---------------------------------------------------------------------------
# Responder side (SURVEY 8f-4 remainder) and cookies
# ---------------------------------------------------------------------------
WRONG_KEY, WRONG_TAI64N_TIMESTAMP = 6, 8  # WireGuardError index + 1
HANDSHAKE_RESP, HANDSHAKE_RESP_SZ, COOKIE_REPLY, COOKIE_REPLY_SZ = 2, 92, 3, 64


def b2s_keyed_mac(key: bytes, data: bytes, n: int) -> bytes:
    """Blake2sMac<n> (keyed BLAKE2s): b2s_keyed_mac_16 / _16_2 / b2s_mac_24 (handshake.rs:74-97)."""
    return hashlib.blake2s(data, key=key, digest_size=n).digest()


def consume_initiation(static_private: bytes, peer_static_public: bytes, static_shared: bytes,
                       msg: bytes):
    """receive_handshake_initialization (handshake.rs:527-613) up to the TAI64N replay
    comparison, which needs the peer's last timestamp (see timestamp_after).
    -> (status, peer_index, timestamp, chaining_key, hash, peer_ephemeral)."""
    static_public = public_key(static_private)
    ck = INITIAL_CHAIN_KEY
    h = b2s_hash(INITIAL_CHAIN_HASH, static_public)
    peer_index = int.from_bytes(msg[4:8], "little")
    eph = msg[8:40]
    h = b2s_hash(h, eph)
    ck = b2s_hmac(b2s_hmac(ck, eph), b"\x01")
    temp = b2s_hmac(ck, x25519(static_private, eph))
    ck = b2s_hmac(temp, b"\x01")
    key = b2s_hmac(temp, ck, b"\x02")
    fail = (bytes(12), bytes(32), bytes(32), bytes(32))
    pt = o.aead_open(key, _nonce0(), h, msg[40:72], msg[72:88])
    if pt is None:
        return (INVALID_AEAD_TAG, peer_index) + fail
    if pt != peer_static_public:
        return (WRONG_KEY, peer_index) + fail
    h = b2s_hash(h, msg[40:88])
    temp = b2s_hmac(ck, static_shared)
    ck = b2s_hmac(temp, b"\x01")
    key = b2s_hmac(temp, ck, b"\x02")
    ts = o.aead_open(key, _nonce0(), h, msg[88:100], msg[100:116])
    if ts is None:
        return (INVALID_AEAD_TAG, peer_index) + fail
    h = b2s_hash(h, msg[88:116])
    return 0, peer_index, ts, ck, h, eph


def timestamp_after(ts: bytes, last: bytes) -> bool:
    """Tai64N::parse + after (handshake.rs:239-269): big-endian secs, then nanos."""
    return (int.from_bytes(ts[:8], "big"), int.from_bytes(ts[8:], "big")) > \
        (int.from_bytes(last[:8], "big"), int.from_bytes(last[8:], "big"))


def format_response(chaining_key: bytes, hsh: bytes, peer_ephemeral: bytes, peer_index: int,
                    local_index: int, ephemeral_private: bytes, peer_static_public: bytes,
                    preshared_key: bytes | None = None, cookie: bytes | None = None):
    """format_handshake_response (handshake.rs:853-949) + append_mac1_and_mac2 (:732-765),
    with the random ephemeral key and inc_index() result supplied.
    -> (response 92 bytes, receiving_key = temp2, sending_key = temp3, mac1)."""
    ck, h = chaining_key, hsh
    eph_pub = public_key(ephemeral_private)
    h = b2s_hash(h, eph_pub)
    temp = b2s_hmac(ck, eph_pub)
    ck = b2s_hmac(temp, b"\x01")
    temp = b2s_hmac(ck, x25519(ephemeral_private, peer_ephemeral))
    ck = b2s_hmac(temp, b"\x01")
    temp = b2s_hmac(ck, x25519(ephemeral_private, peer_static_public))
    ck = b2s_hmac(temp, b"\x01")
    temp = b2s_hmac(ck, preshared_key or bytes(32))
    ck = b2s_hmac(temp, b"\x01")
    temp2 = b2s_hmac(temp, ck, b"\x02")
    key = b2s_hmac(temp, temp2, b"\x03")
    h = b2s_hash(h, temp2)
    ct, tag = o.aead_seal(key, _nonce0(), h, b"")
    msg = (HANDSHAKE_RESP.to_bytes(4, "little") + local_index.to_bytes(4, "little") +
           peer_index.to_bytes(4, "little") + eph_pub + ct + tag)
    t1 = b2s_hmac(ck, b"")
    t2 = b2s_hmac(t1, b"\x01")
    t3 = b2s_hmac(t1, t2, b"\x02")
    mac1 = b2s_keyed_mac_16(b2s_hash(LABEL_MAC1, peer_static_public), msg)
    mac2 = b2s_keyed_mac(cookie, msg + mac1, 16) if cookie else bytes(16)
    return msg + mac1 + mac2, t2, t3, mac1


def hchacha20(key: bytes, nonce16: bytes) -> bytes:
    """HChaCha20 (draft-irtf-cfrg-xchacha-03 2.2): the ChaCha20 rounds without the
    feed-forward, words 0-3 and 12-15 of the state."""
    import struct
    M = 0xFFFFFFFF
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(struct.unpack("<8I", key)) + \
        list(struct.unpack("<4I", nonce16))

    def rotl(x, n):
        return ((x << n) | (x >> (32 - n))) & M

    def qr(a, b, c, d):
        s[a] = (s[a] + s[b]) & M; s[d] = rotl(s[d] ^ s[a], 16)  # noqa: E702
        s[c] = (s[c] + s[d]) & M; s[b] = rotl(s[b] ^ s[c], 12)  # noqa: E702
        s[a] = (s[a] + s[b]) & M; s[d] = rotl(s[d] ^ s[a], 8)  # noqa: E702
        s[c] = (s[c] + s[d]) & M; s[b] = rotl(s[b] ^ s[c], 7)  # noqa: E702
    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)  # noqa: E702
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)  # noqa: E702
    return struct.pack("<8I", *(s[0:4] + s[12:16]))


def xchacha20poly1305_seal(key: bytes, nonce24: bytes, aad: bytes, pt: bytes) -> bytes:
    """XChaCha20-Poly1305 (chacha20poly1305 0.10 XChaCha20Poly1305, rate_limiter.rs:156-164):
    subkey = HChaCha20(key, nonce[:16]), then RFC 8439 with nonce 0^4 || nonce[16:]."""
    ct, tag = o.aead_seal(hchacha20(key, nonce24[:16]), bytes(4) + nonce24[16:], aad, pt)
    return ct + tag


def xchacha20poly1305_open(key: bytes, nonce24: bytes, aad: bytes, ct_tag: bytes) -> bytes | None:
    return o.aead_open(hchacha20(key, nonce24[:16]), bytes(4) + nonce24[16:], aad, ct_tag[:-16],
                       ct_tag[-16:])


def current_cookie(secret_key: bytes, cur_counter: int, addr16: bytes) -> bytes:
    """RateLimiter::current_cookie (rate_limiter.rs:93-110): MAC(secret, LE64(counter) || addr)."""
    return b2s_keyed_mac(secret_key, cur_counter.to_bytes(8, "little") + addr16, 16)


def cookie_nonce(nonce_key: bytes, ctr: int) -> bytes:
    """RateLimiter::nonce (rate_limiter.rs:112-121): b2s_mac_24(nonce_key, LE64(ctr))."""
    return b2s_keyed_mac(nonce_key, ctr.to_bytes(8, "little"), 24)


def mac2_ok(cookie: bytes, msg: bytes) -> bool:
    """verify_packet's under-load mac2 check (rate_limiter.rs:197-210) on a whole
    handshake message (mac1 and mac2 are its last 32 bytes)."""
    return b2s_keyed_mac(cookie, msg[:-16], 16) == msg[-16:]


def format_cookie_reply(cookie_key: bytes, sender_idx: int, cookie: bytes, mac1: bytes,
                        nonce24: bytes) -> bytes:
    """RateLimiter::format_cookie_reply (rate_limiter.rs:133-170)."""
    return (COOKIE_REPLY.to_bytes(4, "little") + sender_idx.to_bytes(4, "little") + nonce24 +
            xchacha20poly1305_seal(cookie_key, nonce24, mac1, cookie))


def receive_response(chaining_key: bytes, hsh: bytes, ephemeral_private: bytes,
                     static_private: bytes, msg: bytes, preshared_key: bytes | None = None):
    """Initiator side, receive_handshake_response (handshake.rs:615-695) from the
    InitSent state of `initiation`.  -> (status, sending_key = temp2, receiving_key = temp3)."""
    eph = msg[12:44]
    h = b2s_hash(hsh, eph)
    temp = b2s_hmac(chaining_key, eph)
    ck = b2s_hmac(temp, b"\x01")
    temp = b2s_hmac(ck, x25519(ephemeral_private, eph))
    ck = b2s_hmac(temp, b"\x01")
    temp = b2s_hmac(ck, x25519(static_private, eph))
    ck = b2s_hmac(temp, b"\x01")
    temp = b2s_hmac(ck, preshared_key or bytes(32))
    ck = b2s_hmac(temp, b"\x01")
    temp2 = b2s_hmac(temp, ck, b"\x02")
    key = b2s_hmac(temp, temp2, b"\x03")
    h = b2s_hash(h, temp2)
    if o.aead_open(key, _nonce0(), h, b"", msg[44:60]) is None:
        return INVALID_AEAD_TAG, bytes(32), bytes(32)
    t1 = b2s_hmac(ck, b"")
    t2 = b2s_hmac(t1, b"\x01")
    t3 = b2s_hmac(t1, t2, b"\x02")
    return 0, t2, t3
