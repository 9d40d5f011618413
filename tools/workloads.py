"""Batch layouts for BASELINE.json configs 2-4 (bench and tests; not the product).

Every layout is NepTUN's slot layout (device/mod.rs:74-76): each packet owns a
slot of round_up(P + 32, 128) bytes, the datagram sits at the slot start and
the plaintext 16 bytes in (WG_HEADER_OFFSET), so encapsulate_in_place-style
batches are 128-byte-run aligned on both sides.
"""
from __future__ import annotations

import numpy as np

from neptun_amd.gpu import DESC_DTYPE
from tools import synth

MIXED_SIZES = (64, 256, 576, 1350, 8900)  # BASELINE config 3


def slot_size(p: int) -> int:
    return synth.round_up(p + 32, 128)


class DescBatch:
    """Descriptor batch on the device: pt buffer (plaintext at slot+16), wire
    buffer (datagram at slot+0), out buffer (recovered plaintext at slot+16)."""

    def __init__(self, sizes: np.ndarray, counters: np.ndarray, slots: np.ndarray, device,
                 seed: int = synth.SEED):
        import torch
        self.n = len(sizes)
        self.sizes = sizes.astype(np.uint32)
        slot = ((self.sizes.astype(np.int64) + 32 + 127) // 128) * 128
        self.offs = np.zeros(self.n, np.int64)
        self.offs[1:] = np.cumsum(slot)[:-1]
        self.total = int(slot.sum())
        seal = np.zeros(self.n, DESC_DTYPE)
        seal["src_off"] = self.offs + 16
        seal["dst_off"] = self.offs
        seal["counter"] = counters
        seal["len"] = self.sizes
        seal["key_slot"] = slots
        opn = np.zeros(self.n, DESC_DTYPE)
        opn["src_off"] = self.offs
        opn["dst_off"] = self.offs + 16
        opn["len"] = self.sizes + 32
        opn["key_slot"] = slots
        self.seal_host, self.open_host = seal, opn
        self.d_seal = torch.from_numpy(seal.view(np.uint8)).to(device)
        self.d_open = torch.from_numpy(opn.view(np.uint8)).to(device)
        g = torch.Generator(device=device)
        g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
        self.pt = torch.randint(0, 256, (self.total + 64,), dtype=torch.uint8, device=device,
                                generator=g)
        self.wire = torch.zeros_like(self.pt)
        self.out = torch.zeros_like(self.pt)
        self.st_seal = torch.full((self.n,), -1, dtype=torch.int32, device=device)
        self.st_open = torch.full((self.n,), -1, dtype=torch.int32, device=device)
        self.order = torch.zeros(self.n, dtype=torch.int32, device=device)
        self.scratch = torch.zeros(262144 // 4, dtype=torch.int32, device=device)  # WG_PLAN_SCRATCH_BYTES

    def round_trip_equal(self, chunk: int = 1 << 14) -> bool:
        """out == pt over every packet's plaintext bytes (chunked gathers, per size)."""
        import torch
        dev = self.pt.device
        for p in np.unique(self.sizes):
            sel = np.nonzero(self.sizes == p)[0]
            ar = torch.arange(int(p), device=dev, dtype=torch.int64)
            for c in range(0, len(sel), chunk):
                starts = torch.from_numpy(self.offs[sel[c:c + chunk]] + 16).to(dev)
                idx = (starts[:, None] + ar[None, :]).reshape(-1)
                if not torch.equal(self.out[idx], self.pt[idx]):
                    return False
        return True

    def sample(self, k: int, keys: np.ndarray, key_index: np.ndarray) -> list:
        """k (key, receiver_idx, counter, payload, datagram) tuples spread over the batch."""
        idx = np.unique(np.linspace(0, self.n - 1, min(k, self.n)).astype(np.int64))
        out = []
        for i in idx:
            d = self.seal_host[i]
            o, P = int(self.offs[i]), int(self.sizes[i])
            pt = self.pt[o + 16:o + 16 + P].cpu().numpy().tobytes()
            wire = self.wire[o:o + P + 32].cpu().numpy().tobytes()
            slot = int(d["key_slot"])
            out.append((keys[slot].tobytes(), int(key_index[slot]), int(d["counter"]), pt, wire))
        return out


def config3(per_size: int, device, seed: int = synth.SEED, sizes=MIXED_SIZES) -> DescBatch:
    """{64,256,576,1350,8900} x per_size, seeded interleave, one session (counters 0..n-1)."""
    rng = np.random.default_rng(seed)
    sizes = np.repeat(np.array(sizes, np.uint32), per_size)
    sizes = sizes[rng.permutation(len(sizes))]
    n = len(sizes)
    return DescBatch(sizes, np.arange(n, dtype=np.uint64), np.zeros(n, np.uint32), device, seed)


def config4(peers: int, per_peer: int, size: int, device, seed: int = synth.SEED) -> DescBatch:
    """peers x per_peer packets of `size` bytes; packet -> peer by a seeded permutation
    (neighbouring lanes hit different keys); per-peer counters run 0..per_peer-1."""
    rng = np.random.default_rng(seed)
    n = peers * per_peer
    peer = (rng.permutation(n) % peers).astype(np.uint32)
    # counter = rank of the packet among its peer's packets, in batch order
    order = np.argsort(peer, kind="stable")
    ctr = np.empty(n, np.uint64)
    ctr[order] = np.tile(np.arange(per_peer, dtype=np.uint64), peers)
    return DescBatch(np.full(n, size, np.uint32), ctr, peer, device, seed)
