"""ctypes wrapper over oracle/build/libneptun_oracle.so -- TEST INFRASTRUCTURE ONLY.

Restates NepTUN's transport-data seal/open (neptun/src/noise/session.rs:205-302)
over RFC 8439 ChaCha20-Poly1305 (ring 0.17.14's algorithm); see
oracle/neptun_oracle.c for the per-function citations.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "build")

DATA_OFFSET = 16          # session.rs:31
AEAD_SIZE = 16            # session.rs:33
DATA_OVERHEAD_SZ = 32     # noise/mod.rs:91
MSG_DATA = 4              # noise/mod.rs:86

# numpy view of neptun_oracle_desc / wg_packet_desc (32 bytes)
DESC_DTYPE = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("counter", "<u8"),
                       ("len", "<u4"), ("key_slot", "<u4")])
assert DESC_DTYPE.itemsize == 32


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load(name: str) -> ctypes.CDLL:
    path = os.path.join(_BUILD, name)
    if not os.path.exists(path):
        build()
    return ctypes.CDLL(path)


_lib = None
_ossl = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = _load("libneptun_oracle.so")
        c = ctypes
        u8p = c.c_char_p
        L.neptun_oracle_chacha20_block.argtypes = [u8p, c.c_uint32, u8p, c.c_void_p]
        L.neptun_oracle_poly1305.argtypes = [u8p, u8p, c.c_size_t, c.c_void_p]
        L.neptun_oracle_aead_seal.argtypes = [u8p, u8p, u8p, c.c_size_t, u8p, c.c_size_t,
                                              c.c_void_p, c.c_void_p]
        L.neptun_oracle_aead_open.argtypes = [u8p, u8p, u8p, c.c_size_t, u8p, c.c_size_t, u8p,
                                              c.c_void_p]
        L.neptun_oracle_format_packet_data.argtypes = [u8p, c.c_uint32, c.c_uint64, u8p,
                                                       c.c_size_t, c.c_void_p, c.c_size_t]
        L.neptun_oracle_receive_packet_data.argtypes = [u8p, c.c_uint32, u8p, c.c_size_t,
                                                        c.c_void_p, c.c_size_t,
                                                        c.POINTER(c.c_size_t)]
        for fn in (L.neptun_oracle_seal_batch, L.neptun_oracle_open_batch):
            fn.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p, c.c_void_p,
                           c.c_void_p, c.c_void_p]
            fn.restype = None
        _lib = L
    return _lib


def openssl() -> ctypes.CDLL:
    """Independent RFC 8439 implementation (OpenSSL 3 EVP) for cross-checks."""
    global _ossl
    if _ossl is None:
        L = _load("libneptun_openssl_ref.so")
        c = ctypes
        u8p = c.c_char_p
        L.ossl_aead_seal.argtypes = [u8p, u8p, u8p, c.c_int, u8p, c.c_int, c.c_void_p, c.c_void_p]
        L.ossl_aead_open.argtypes = [u8p, u8p, u8p, c.c_int, u8p, c.c_int, u8p, c.c_void_p]
        L.ossl_format_packet_data.argtypes = [u8p, c.c_uint32, c.c_uint64, u8p, c.c_int, c.c_void_p]
        L.ossl_receive_packet_data.argtypes = [u8p, u8p, c.c_int, c.c_void_p]
        L.ossl_x25519.argtypes = [c.c_void_p, u8p, u8p]
        _ossl = L
    return _ossl


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().neptun_oracle_chacha20_block(key, counter, nonce, out)
    return out.raw


def poly1305(key: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(16)
    lib().neptun_oracle_poly1305(key, msg, len(msg), out)
    return out.raw


def aead_seal(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    ct = ctypes.create_string_buffer(max(len(pt), 1))
    tag = ctypes.create_string_buffer(16)
    lib().neptun_oracle_aead_seal(key, nonce, aad, len(aad), pt, len(pt), ct, tag)
    return ct.raw[: len(pt)], tag.raw


def aead_open(key: bytes, nonce: bytes, aad: bytes, ct: bytes, tag: bytes) -> bytes | None:
    pt = ctypes.create_string_buffer(max(len(ct), 1))
    rc = lib().neptun_oracle_aead_open(key, nonce, aad, len(aad), ct, len(ct), tag, pt)
    return None if rc else pt.raw[: len(ct)]


def format_packet_data(key: bytes, sending_index: int, counter: int, payload: bytes) -> bytes:
    """Session::format_packet_data (session.rs:205-259): returns the wire packet."""
    out = ctypes.create_string_buffer(len(payload) + DATA_OVERHEAD_SZ)
    rc = lib().neptun_oracle_format_packet_data(key, sending_index, counter, payload,
                                                len(payload), out, len(out))
    assert rc == 0
    return out.raw


def receive_packet_data(key: bytes, receiving_index: int, datagram: bytes) -> tuple[int, bytes]:
    """Session::receive_packet_data (session.rs:265-302, no replay window).

    Returns (status, plaintext); status 0 = Ok, else WireGuardError index + 1.
    """
    cap = max(len(datagram) - DATA_OFFSET, 1)
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    rc = lib().neptun_oracle_receive_packet_data(key, receiving_index, datagram, len(datagram),
                                                 out, cap, ctypes.byref(n))
    return rc, out.raw[: n.value]


def seal_batch(descs: np.ndarray, keys: np.ndarray, key_index: np.ndarray, src: np.ndarray,
               dst: np.ndarray) -> np.ndarray:
    status = np.zeros(len(descs), dtype=np.int32)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    key_index = np.ascontiguousarray(key_index, dtype=np.uint32)
    lib().neptun_oracle_seal_batch(descs.ctypes.data, len(descs), keys.ctypes.data,
                                   key_index.ctypes.data, src.ctypes.data, dst.ctypes.data,
                                   status.ctypes.data)
    return status


def open_batch(descs: np.ndarray, keys: np.ndarray, key_index: np.ndarray, src: np.ndarray,
               dst: np.ndarray) -> np.ndarray:
    status = np.zeros(len(descs), dtype=np.int32)
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    key_index = np.ascontiguousarray(key_index, dtype=np.uint32)
    lib().neptun_oracle_open_batch(descs.ctypes.data, len(descs), keys.ctypes.data,
                                   key_index.ctypes.data, src.ctypes.data, dst.ctypes.data,
                                   status.ctypes.data)
    return status


def openssl_x25519(scalar: bytes, point: bytes) -> bytes | None:
    """X25519 through OpenSSL (None when OpenSSL rejects an all-zero result)."""
    out = ctypes.create_string_buffer(32)
    return None if openssl().ossl_x25519(out, scalar, point) else out.raw
