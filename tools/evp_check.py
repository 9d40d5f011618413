"""Independent known-answer check for bench.py: OpenSSL 3 EVP_chacha20_poly1305
through ctypes, framed as NepTUN frames a data packet (session.rs:221-246:
LE32 4 | LE32 receiver_idx | LE64 counter | ciphertext | tag, nonce
0^4 || LE64(counter), empty AAD).

Not the oracle (oracle/ is the test suite's checker): this is a third-party
RFC 8439 implementation used by bench.py to compare a sample of the timed
batch's sealed datagrams byte for byte, so a bug that seal and open share
(nonce layout, counter, keystream block index) cannot pass as a round trip.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import struct

_EVP_CTRL_AEAD_SET_IVLEN = 0x9
_EVP_CTRL_AEAD_GET_TAG = 0x10


class Evp:
    def __init__(self):
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        self.lib = lib = ctypes.CDLL(name)
        lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        lib.EVP_chacha20_poly1305.restype = ctypes.c_void_p
        lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_char_p, ctypes.c_char_p]
        lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                          ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        lib.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                            ctypes.POINTER(ctypes.c_int)]
        lib.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

    def seal_datagram(self, key: bytes, receiver_idx: int, counter: int, payload: bytes) -> bytes:
        lib = self.lib
        ctx = lib.EVP_CIPHER_CTX_new()
        if not ctx:
            raise RuntimeError("EVP_CIPHER_CTX_new failed")
        try:
            nonce = b"\0" * 4 + struct.pack("<Q", counter)
            ok = lib.EVP_EncryptInit_ex(ctx, lib.EVP_chacha20_poly1305(), None, None, None)
            ok &= lib.EVP_CIPHER_CTX_ctrl(ctx, _EVP_CTRL_AEAD_SET_IVLEN, 12, None)
            ok &= lib.EVP_EncryptInit_ex(ctx, None, None, key, nonce)
            out = ctypes.create_string_buffer(len(payload) + 16)
            n = ctypes.c_int(0)
            if payload:
                ok &= lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), payload, len(payload))
            m = ctypes.c_int(0)
            ok &= lib.EVP_EncryptFinal_ex(ctx, ctypes.cast(ctypes.byref(out, n.value), ctypes.c_char_p),
                                          ctypes.byref(m))
            tag = ctypes.create_string_buffer(16)
            ok &= lib.EVP_CIPHER_CTX_ctrl(ctx, _EVP_CTRL_AEAD_GET_TAG, 16, tag)
            if ok != 1:
                raise RuntimeError("EVP chacha20-poly1305 failed")
            header = struct.pack("<IIQ", 4, receiver_idx, counter)
            return header + out.raw[:n.value + m.value] + tag.raw
        finally:
            lib.EVP_CIPHER_CTX_free(ctx)
