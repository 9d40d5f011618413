"""Batched handshake kernels (wg_handshake.hip) vs the oracle:
X25519 (RFC 7748 vectors, random and edge-case points) and the responder's
pre-peer work on handshake initiations: mac1 (rate_limiter.rs:187-195) +
parse_handshake_anon (handshake.rs:367-412)."""
import json
import os
import random

import numpy as np
import pytest

from oracle import handshake_model as H

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "handshake.json")))


def to_dev(torch, b: bytes):
    return torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()


def test_x25519_batch_matches_oracle(torch_cuda, gpu):
    torch = torch_cuda
    rng = random.Random(13)
    p = H.P25519
    scal, pts = [], []
    v = GOLDEN["scalarmult"][0]
    scal.append(bytes.fromhex(v["scalar"]))
    pts.append(bytes.fromhex(v["u"]))
    d = GOLDEN["dh"]
    scal += [bytes.fromhex(d["alice_private"]), bytes.fromhex(d["bob_private"])]
    pts += [bytes.fromhex(d["bob_public"]), (9).to_bytes(32, "little")]
    for x in (0, 1, p - 1, p, p + 1, 2**255 - 1, 2**256 - 1):
        scal.append(rng.randbytes(32))
        pts.append((x % 2**256).to_bytes(32, "little"))
    while len(scal) < 700:  # > 2 workgroups, ragged tail
        scal.append(rng.randbytes(32))
        pts.append(rng.randbytes(32))
    n = len(scal)
    d_s, d_p = to_dev(torch, b"".join(scal)), to_dev(torch, b"".join(pts))
    d_o = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    gpu.x25519_batch(n, d_s, d_p, d_o)
    torch.cuda.synchronize()
    out = d_o.cpu().numpy().tobytes()
    for i in range(n):
        assert out[32 * i:32 * i + 32] == H.x25519(scal[i], pts[i]), i
    assert out[:32].hex() == v["out"]
    assert out[64:96].hex() == d["bob_public"]


def test_handshake_anon_batch_matches_oracle(torch_cuda, gpu):
    from neptun_amd.gpu import HALF_HANDSHAKE_DTYPE
    torch = torch_cuda
    rng = random.Random(17)
    resp_priv = rng.randbytes(32)
    resp_pub = H.public_key(resp_priv)
    msgs, kinds = [], []
    for i in range(300):
        init_priv = rng.randbytes(32)
        m = bytearray(H.format_handshake_initiation(init_priv, resp_pub, rng.randbytes(32),
                                                    rng.getrandbits(32), rng.randbytes(12)))
        r = rng.random()
        if r < 0.1:
            m[rng.randrange(0, 116)] ^= 1 << rng.randrange(8)   # mac1 fails
        elif r < 0.2:
            m[rng.randrange(116, 132)] ^= 1                      # the mac1 bytes themselves
        elif r < 0.25:
            m[0] = 2                                             # not an initiation
        elif r < 0.3:
            other = H.public_key(rng.randbytes(32))              # sent to someone else
            m = bytearray(H.format_handshake_initiation(init_priv, other, rng.randbytes(32), 5,
                                                        rng.randbytes(12)))
        msgs.append(bytes(m))
    stride = 152
    buf = b"".join(m + bytes(stride - len(m)) for m in msgs)
    d_m = to_dev(torch, buf)
    for check_mac1 in (True, False):
        d_o = torch.zeros(len(msgs) * HALF_HANDSHAKE_DTYPE.itemsize, dtype=torch.uint8,
                          device="cuda")
        gpu.handshake_anon_batch(resp_priv, len(msgs), d_m, stride, d_o, check_mac1=check_mac1)
        torch.cuda.synchronize()
        res = d_o.cpu().numpy().view(HALF_HANDSHAKE_DTYPE)
        for i, m in enumerate(msgs):
            st, idx, pub = H.parse_handshake_anon(resp_priv, resp_pub, m, check_mac1)
            assert res[i]["status"] == st, (i, check_mac1, res[i]["status"], st)
            if st == 0:
                assert res[i]["peer_index"] == idx
                assert res[i]["peer_static_public"].tobytes() == pub
        sts = {int(x) for x in res["status"]}
        # with mac1 on, every damaged message fails mac1 first; without it, the AEAD
        assert sts == ({0, H.INVALID_MAC, H.WRONG_PACKET_TYPE} if check_mac1 else
                       {0, H.INVALID_AEAD_TAG, H.WRONG_PACKET_TYPE})
