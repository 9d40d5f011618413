"""Split waves of the strided batches (wg_gpu_ctx_set_split; wg_aead.hip
aead_strided_split_kernel + aead_strided_finish_kernel): each wave of 64 packets runs
as K jobs over consecutive rounds, a finish kernel combines their Poly1305 sums.

Every byte of the destination buffers -- packets, slot padding and the canaries around
them -- and every status must equal the unsplit kernels' (K = 1) and, on sampled
packets, the oracle (oracle/neptun_oracle.c: session.rs:205-302 + RFC 8439): seal, and
open on the wire grid and on the text grid (NepTUN's own layout) with tampered
ciphertext / tags (ring's zeros), foreign headers and wrong receiver indices.  Sizes
cover whole and partial tail chunks and tags straddling two rounds; the BASELINE AEAD
bench size 8192 B (chacha20poly1305_benching.rs:37-55) at every K.
"""
import numpy as np
import pytest

from oracle import pyoracle as o
from tools import synth

pytestmark = pytest.mark.gpu

KIDX = 0x2468ACE1
# (payload, K with parts of >= 8 keystream rounds; K that do not divide the rounds
# give part 0 the remainder)
CASES = [(8192, 2), (8192, 3), (8192, 4), (8192, 5), (8192, 7), (8192, 8), (8190, 4), (8177, 6), (8177, 8),
         (4096, 2), (4096, 3), (4000, 4), (2048, 2)]


@pytest.fixture
def split_ctx(gpu):
    yield gpu
    gpu.set_split(-1)
    gpu.set_slot_padding(False)


def _seal(torch, ctx, K, n, P, S, src, pad, ctr0):
    ctx.set_split(K)
    ctx.set_slot_padding(pad)
    w = torch.full((n * S + 256,), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ctx.seal_strided(n, P, 0, ctr0, src.data_ptr() + 16, S, w, S, st)
    torch.cuda.synchronize()
    return w, st


@pytest.mark.parametrize("pad", [False, True])
@pytest.mark.parametrize("P,K", CASES)
def test_split_seal_equals_unsplit_and_oracle(torch_cuda, split_ctx, P, K, pad):
    torch = torch_cuda
    ctx = split_ctx
    rng = np.random.default_rng(P * 16 + K + pad)
    key = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    ctx.set_keys(0, key, np.array([KIDX], np.uint32))
    n, S = 64 * 5 + 9, synth.round_up(P + 32, 128)
    src = torch.from_numpy(rng.integers(0, 256, n * S + 256, dtype=np.uint8)).cuda()
    ctr0 = 2**32 - 130
    w1, st1 = _seal(torch, ctx, 1, n, P, S, src, pad, ctr0)
    wk, stk = _seal(torch, ctx, K, n, P, S, src, pad, ctr0)
    assert (st1.cpu().numpy() == 0).all() and (stk.cpu().numpy() == 0).all()
    assert torch.equal(w1, wk), "split seal differs from the unsplit kernels"
    got, s_np = wk.cpu().numpy(), src.cpu().numpy()
    for i in (0, 63, 64, 127, 200, 319, n - 1):
        want = o.format_packet_data(key[0].tobytes(), KIDX, ctr0 + i, s_np[i * S + 16:i * S + 16 + P].tobytes())
        assert got[i * S:i * S + P + 32].tobytes() == want, i


@pytest.mark.parametrize("grid", ["wire", "text"])
@pytest.mark.parametrize("P,K", CASES)
def test_split_open_equals_unsplit_with_failures(torch_cuda, split_ctx, P, K, grid):
    torch = torch_cuda
    ctx = split_ctx
    rng = np.random.default_rng(P * 32 + K + (grid == "text"))
    key = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    ctx.set_keys(0, key, np.array([KIDX], np.uint32))
    n, S = 64 * 5 + 9, synth.round_up(P + 32, 128)
    src = torch.from_numpy(rng.integers(0, 256, n * S + 256, dtype=np.uint8)).cuda()
    wire, st = _seal(torch, ctx, 1, n, P, S, src, False, 7)
    assert (st.cpu().numpy() == 0).all()
    w = wire.cpu().numpy()
    damaged = {}
    for i in rng.choice(n - 9, 40, replace=False):  # (full waves: the tail is never split)
        i = int(i)
        kind = i % 4
        if kind == 0:
            w[i * S + 16 + int(rng.integers(P))] ^= 1 << int(rng.integers(8))  # ciphertext
            damaged[i] = 10
        elif kind == 1:
            w[i * S + 16 + P + int(rng.integers(16))] ^= 0x40  # tag
            damaged[i] = 10
        elif kind == 2:
            w[i * S] = 1  # a handshake type
            damaged[i] = 13
        else:
            w[i * S + 4] ^= 0x10  # receiver index
            damaged[i] = 5
    wire_d = torch.from_numpy(w).cuda()
    off = 0 if grid == "text" else 16  # text grid: plaintext slots on 128-byte lines
    outs = []
    for k in (1, K):
        ctx.set_split(k)
        back = torch.full((n * S + 256,), 0x5A, dtype=torch.uint8, device="cuda")
        st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        ctx.open_strided(n, P + 32, 0, wire_d, S, back.data_ptr() + off, S, st)
        torch.cuda.synchronize()
        outs.append((back.cpu().numpy(), st.cpu().numpy()))
    (b1, s1), (bk, sk) = outs
    assert (s1 == sk).all(), "split open statuses differ"
    assert np.array_equal(b1, bk), "split open bytes differ"
    want = np.zeros(n, np.int32)
    for i, c in damaged.items():
        want[i] = c
    assert (sk == want).all(), (sk[sk != want], want[sk != want])
    s_np = src.cpu().numpy()
    for i in range(n):
        p = bk[i * S + off:i * S + off + P]
        if want[i] == 0:
            assert p.tobytes() == s_np[i * S + 16:i * S + 16 + P].tobytes(), i
        elif want[i] == 10:
            assert not p.any(), i  # ring's open_within leaves zeros
        else:
            assert (p == 0x5A).all(), i  # header failures write nothing


def test_split_choice_fills_the_grid(torch_cuda, split_ctx):
    """The default choice splits the reference bench's 8192-byte batch (172,544
    packets: 2,696 waves on a 4,096-slot grid) and leaves the headline's 1350-byte one
    (16,384 waves) alone -- both bit-exact against the unsplit kernels."""
    torch = torch_cuda
    ctx = split_ctx
    rng = np.random.default_rng(5)
    key = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    ctx.set_keys(0, key, np.array([KIDX], np.uint32))
    for P, n in ((8192, 172544), (1350, 1 << 20)):
        S = synth.round_up(P + 32, 128)
        src = synth.device_payloads(n, P, S, "cuda", seed=3, offset=16)
        w1, _ = _seal(torch, ctx, 1, n, P, S, src, True, 0)
        wd, st = _seal(torch, ctx, -1, n, P, S, src, True, 0)
        assert int((st != 0).sum()) == 0
        assert torch.equal(w1, wd), P
        del w1, wd, src


@pytest.mark.parametrize("K", [3, 7])
def test_split_parts_of_unequal_length_share_workgroups(torch_cuda, split_ctx, K):
    """203 waves of 8192-byte packets at K = 3 / 7: more jobs than the grid's 512
    workgroups, so workgroups take 2-3 consecutive jobs and some straddle a part
    boundary -- part 0 (22 / 10 rounds) beside part 1 (21 / 9) in one workgroup.
    Seal and the wire-grid open equal the unsplit kernels' byte for byte."""
    torch = torch_cuda
    ctx = split_ctx
    rng = np.random.default_rng(100 + K)
    key = rng.integers(0, 256, (1, 32), dtype=np.uint8)
    ctx.set_keys(0, key, np.array([KIDX], np.uint32))
    P, n = 8192, 64 * 203
    S = synth.round_up(P + 32, 128)
    src = synth.device_payloads(n, P, S, "cuda", seed=11 + K, offset=16)
    w1, st1 = _seal(torch, ctx, 1, n, P, S, src, False, 99)
    wk, stk = _seal(torch, ctx, K, n, P, S, src, False, 99)
    assert int((st1 != 0).sum()) == 0 and int((stk != 0).sum()) == 0
    assert torch.equal(w1, wk), "split seal differs from the unsplit kernels"
    got, s_np = wk.cpu().numpy(), src.cpu().numpy()
    for i in (0, 203 * 32 + 5, n - 1):
        want = o.format_packet_data(key[0].tobytes(), KIDX, 99 + i, s_np[i * S + 16:i * S + 16 + P].tobytes())
        assert got[i * S:i * S + P + 32].tobytes() == want, i
    ctx.set_split(K)
    back = torch.full((n * S + 256,), 0x5A, dtype=torch.uint8, device="cuda")
    st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    ctx.open_strided(n, P + 32, 0, wk, S, back.data_ptr() + 16, S, st)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    b = back[: n * S].view(n, S)
    assert torch.equal(b[:, 16:16 + P], src[: n * S].view(n, S)[:, 16:16 + P])
