#!/usr/bin/env python3
"""Golden vectors for the cookie AEAD (XChaCha20-Poly1305, rate_limiter.rs:156-164 /
handshake.rs:719) -- TEST INFRASTRUCTURE.  The reference's XChaCha comes from the
RustCrypto chacha20poly1305 0.10.1 crate (Cargo.lock), which is not vendored; the
vectors are produced here by an independent implementation, libsodium's
crypto_aead_xchacha20poly1305_ietf_encrypt / crypto_core_hchacha20 (/opt/conda),
plus the HChaCha20 test vector of draft-irtf-cfrg-xchacha-03 section 2.2.1.
Writes tests/golden/xchacha.json."""
import ctypes
import json
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    L = ctypes.CDLL("/opt/conda/lib/libsodium.so")
    assert L.sodium_init() >= 0
    rng = random.Random(0x5EED)

    def seal(key, nonce, aad, pt):
        out = ctypes.create_string_buffer(len(pt) + 16)
        ol = ctypes.c_ulonglong()
        L.crypto_aead_xchacha20poly1305_ietf_encrypt(out, ctypes.byref(ol), pt, ctypes.c_ulonglong(len(pt)),
                                                     aad, ctypes.c_ulonglong(len(aad)), None, nonce, key)
        return out.raw[:ol.value]

    def hchacha(key, n16):
        out = ctypes.create_string_buffer(32)
        L.crypto_core_hchacha20(out, n16, key, None)
        return out.raw

    vecs = []
    for i in range(24):
        key, nonce = rng.randbytes(32), rng.randbytes(24)
        aad = rng.randbytes(16 if i % 2 == 0 else rng.randrange(0, 40))
        pt = rng.randbytes(16 if i % 3 == 0 else rng.randrange(0, 80))
        vecs.append({"key": key.hex(), "nonce": nonce.hex(), "aad": aad.hex(), "pt": pt.hex(),
                     "ct_tag": seal(key, nonce, aad, pt).hex(),
                     "hchacha20_subkey": hchacha(key, nonce[:16]).hex()})
    doc = {"source": "libsodium (conda) crypto_aead_xchacha20poly1305_ietf_encrypt, "
                     "crypto_core_hchacha20; draft-irtf-cfrg-xchacha-03 2.2.1",
           "hchacha20_draft": {"key": bytes(range(32)).hex(), "nonce": "000000090000004a0000000031415927",
                               "subkey": "82413b4227b27bfed30e42508a877d73a0f9e4d58a74a853c12ec41326d3ecdc"},
           "vectors": vecs}
    with open(os.path.join(ROOT, "tests", "golden", "xchacha.json"), "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
