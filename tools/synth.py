"""Synthetic packet batches for tests and bench.py (not part of the product).

Payloads follow BASELINE.md: each plaintext is a valid IPv4 header (ver 4,
IHL 5, total_length = P, proto 17, 10.0.0.1 -> 10.0.0.2) followed by seeded
PRNG bytes, so validate_decapsulated_packet (noise/mod.rs:613-634) keeps all P
bytes.  Generated on the device with a seeded torch generator (bit-identical
for a given seed, size and device), so 1M x 1350 B never crosses PCIe.
"""
from __future__ import annotations

import numpy as np

SEED = 0x4E455054554E  # "NEPTUN"
RECEIVER_IDX = 0x00ABCD01


def round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n uint64 values of splitmix64 (vectorised)."""
    s = (np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
    z = s
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def keys(n: int, seed: int = SEED + 1) -> np.ndarray:
    return splitmix64(seed, 4 * n).view(np.uint8).reshape(n, 32).copy()


def ipv4_header(total_len: int) -> bytes:
    h = bytearray(20)
    h[0] = 0x45
    h[2:4] = total_len.to_bytes(2, "big")
    h[8] = 64
    h[9] = 17
    h[12:16] = bytes([10, 0, 0, 1])
    h[16:20] = bytes([10, 0, 0, 2])
    return bytes(h)


def device_payloads(n: int, size: int, stride: int, device, seed: int = SEED, offset: int = 0):
    """uint8 tensor [n * stride] with n plaintexts of `size` bytes at stride.

    Plaintext i occupies [i*stride + offset, i*stride + offset + size); offset 16
    is NepTUN's in-place layout (WG_HEADER_OFFSET, device/mod.rs:76)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    buf = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device=device, generator=g)
    if size >= 20:
        hdr = torch.tensor(list(ipv4_header(size)), dtype=torch.uint8, device=device)
        buf[:, offset:offset + 20] = hdr
    return buf.reshape(-1)


def host_payloads(sizes: np.ndarray, seed: int = SEED) -> list[bytes]:
    rng = np.random.default_rng(seed)
    out = []
    for s in sizes:
        b = bytearray(rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
        if s >= 20:
            b[:20] = ipv4_header(int(s))
        out.append(bytes(b))
    return out
