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


def test_responder_consume_and_respond_match_oracle(torch_cuda, gpu):
    """receive_handshake_initialization (handshake.rs:527-613) on the device, the
    host's TAI64N / inc_index step, then format_handshake_response + mac1/mac2
    (:853-949, :732-765) on the device, vs the oracle -- and the initiators (oracle
    receive_response) accept the responses and derive the same session keys."""
    from neptun_amd import gpu as G
    torch = torch_cuda
    rng = random.Random(29)
    resp_priv = rng.randbytes(32)
    resp_pub = H.public_key(resp_priv)
    n = 300
    inits, peers, msgs, want_status = [], np.zeros(n, G.RESPONDER_PEER_DTYPE), [], []
    for i in range(n):
        si, ei = rng.randbytes(32), rng.randbytes(32)
        pi = H.public_key(si)
        ts = rng.randbytes(12)
        m, ck_i, h_i = H.initiation(si, resp_pub, ei, rng.getrandbits(32), ts)
        m = bytearray(m)
        configured = pi
        r = rng.random()
        if r < 0.05:
            m[rng.randrange(40, 88)] ^= 1          # encrypted static damaged
        elif r < 0.10:
            m[rng.randrange(88, 116)] ^= 1         # encrypted timestamp damaged
        elif r < 0.15:
            configured = H.public_key(rng.randbytes(32))  # not the peer the caller looked up
        elif r < 0.17:
            m[0] = 2
        peers[i]["peer_static_public"] = np.frombuffer(configured, np.uint8)
        peers[i]["static_shared"] = np.frombuffer(H.x25519(resp_priv, configured), np.uint8)
        msgs.append(bytes(m))
        inits.append((si, ei, ck_i, h_i, pi))
    stride = 148
    d_m = to_dev(torch, b"".join(msgs))
    d_p = to_dev(torch, peers.tobytes())
    d_s = torch.zeros(n * G.INIT_RECEIVED_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    gpu.handshake_consume_batch(resp_priv, n, d_m, stride, d_p, d_s)
    torch.cuda.synchronize()
    states = d_s.cpu().numpy().view(G.INIT_RECEIVED_DTYPE)
    jobs = np.zeros(n, G.RESPONSE_JOB_DTYPE)
    oracle_states = []
    last = bytes(12)
    for i, m in enumerate(msgs):
        pub = peers[i]["peer_static_public"].tobytes()
        if m[:4] != b"\x01\x00\x00\x00":
            want = (H.WRONG_PACKET_TYPE, 0)
        else:
            want = H.consume_initiation(resp_priv, pub, H.x25519(resp_priv, pub), m)
        assert int(states[i]["status"]) == want[0], (i, int(states[i]["status"]), want[0])
        oracle_states.append(want)
        if want[0] == 0:
            _, idx, ts, ck, h, eph = want
            assert int(states[i]["peer_index"]) == idx
            assert states[i]["timestamp"].tobytes() == ts
            assert states[i]["chaining_key"].tobytes() == ck and states[i]["hash"].tobytes() == h
            assert states[i]["peer_ephemeral"].tobytes() == eph
            # host step (packet order): every initiator is a different peer here
            assert gpu.timestamp_after(ts, last) == H.timestamp_after(ts, last)
        jobs[i]["ephemeral_private"] = np.frombuffer(rng.randbytes(32), np.uint8)
        jobs[i]["peer_static_public"] = peers[i]["peer_static_public"]
        jobs[i]["preshared_key"] = np.frombuffer(rng.randbytes(32) if i % 3 == 0 else bytes(32), np.uint8)
        jobs[i]["mac1_key"] = np.frombuffer(H.b2s_hash(H.LABEL_MAC1, pub), np.uint8)
        jobs[i]["has_cookie"] = 1 if i % 4 == 0 else 0
        jobs[i]["cookie"] = np.frombuffer(rng.randbytes(16), np.uint8)
        jobs[i]["local_index"] = 0x00ABC000 + i
    assert {s[0] for s in oracle_states} >= {0, H.INVALID_AEAD_TAG, H.WRONG_KEY, H.WRONG_PACKET_TYPE}
    d_j = to_dev(torch, jobs.tobytes())
    d_o = torch.zeros(n * G.RESPONSE_OUT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    gpu.handshake_respond_batch(n, d_s, d_j, d_o)
    torch.cuda.synchronize()
    out = d_o.cpu().numpy().view(G.RESPONSE_OUT_DTYPE)
    accepted = 0
    for i, want in enumerate(oracle_states):
        if want[0] != 0:
            assert not out[i]["message"].any()
            continue
        _, idx, ts, ck, h, eph = want
        j = jobs[i]
        psk = j["preshared_key"].tobytes()
        cookie = j["cookie"].tobytes() if j["has_cookie"] else None
        resp, rk, sk, mac1 = H.format_response(ck, h, eph, idx, int(j["local_index"]),
                                               j["ephemeral_private"].tobytes(),
                                               j["peer_static_public"].tobytes(),
                                               psk if any(psk) else None, cookie)
        assert out[i]["message"].tobytes() == resp, i
        assert out[i]["receiving_key"].tobytes() == rk and out[i]["sending_key"].tobytes() == sk
        assert out[i]["mac1"].tobytes() == mac1
        si, ei, ck_i, h_i, pi = inits[i]
        st, send_i, recv_i = H.receive_response(ck_i, h_i, ei, si, resp, psk if any(psk) else None)
        assert st == 0 and send_i == rk and recv_i == sk
        accepted += 1
    assert accepted > 200


def test_cookie_mac2_check_and_reply_match_oracle(torch_cuda, gpu):
    """Under load (rate_limiter.rs:197-218): cookie from (secret, counter, address),
    mac2 check of initiations and responses, and COOKIE_REPLY messages
    (XChaCha20-Poly1305, :133-170) -- each equal to the oracle, and the initiator
    can open its cookie (receive_cookie_reply, handshake.rs:703-727)."""
    torch = torch_cuda
    rng = random.Random(37)
    secret, nonce_key = rng.randbytes(16), rng.randbytes(32)
    resp_pub = H.public_key(rng.randbytes(32))
    cookie_key = H.b2s_hash(H.LABEL_COOKIE, resp_pub)
    counter = rng.getrandbits(40)
    n = 400
    msgs, lens, addrs, good = [], [], [], []
    for i in range(n):
        addr = rng.randbytes(4) + bytes(12) if i % 2 else rng.randbytes(16)
        ck = H.current_cookie(secret, counter, addr)
        has = rng.random() < 0.5
        if i % 3:
            m = H.format_handshake_initiation(rng.randbytes(32), resp_pub, rng.randbytes(32),
                                              rng.getrandbits(32), rng.randbytes(12),
                                              cookie=ck if has else None)
        else:  # a handshake response-sized message with the macs at its end
            body = rng.randbytes(60)
            mac1 = rng.randbytes(16)
            m = body + mac1 + (H.b2s_keyed_mac(ck, body + mac1, 16) if has else rng.randbytes(16))
        msgs.append(m)
        lens.append(len(m))
        addrs.append(addr)
        good.append(H.mac2_ok(ck, m))
    stride = 148
    d_m = to_dev(torch, b"".join(m + bytes(stride - len(m)) for m in msgs))
    d_l = to_dev(torch, np.array(lens, np.uint32).tobytes())
    d_a = to_dev(torch, b"".join(addrs))
    d_c = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.mac2_check_batch(secret, counter, n, d_m, stride, d_l, d_a, d_c, d_st)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    cookies = d_c.cpu().numpy().tobytes()
    for i in range(n):
        assert cookies[16 * i:16 * i + 16] == H.current_cookie(secret, counter, addrs[i])
        assert st[i] == (0 if good[i] else 1), i
    assert 0 < int(st.sum()) < n
    # replies for the failures, nonce counters handed out in order
    from neptun_amd import gpu as G
    bad = [i for i in range(n) if not good[i]]
    jobs = np.zeros(len(bad), G.COOKIE_REPLY_JOB_DTYPE)
    ctr0 = rng.getrandbits(48)
    for k, i in enumerate(bad):
        jobs[k]["cookie"] = np.frombuffer(cookies[16 * i:16 * i + 16], np.uint8)
        jobs[k]["mac1"] = np.frombuffer(msgs[i][-32:-16], np.uint8)
        jobs[k]["nonce_ctr"] = ctr0 + k
        jobs[k]["receiver_idx"] = int.from_bytes(msgs[i][4:8], "little")
    d_j = to_dev(torch, jobs.tobytes())
    d_o = torch.zeros(64 * len(bad), dtype=torch.uint8, device="cuda")
    gpu.cookie_reply_batch(cookie_key, nonce_key, len(bad), d_j, d_o)
    torch.cuda.synchronize()
    out = d_o.cpu().numpy().tobytes()
    for k, i in enumerate(bad):
        want = H.format_cookie_reply(cookie_key, int(jobs[k]["receiver_idx"]), jobs[k]["cookie"].tobytes(),
                                     jobs[k]["mac1"].tobytes(), H.cookie_nonce(nonce_key, ctr0 + k))
        got = out[64 * k:64 * k + 64]
        assert got == want, k
        assert H.xchacha20poly1305_open(cookie_key, got[8:32], msgs[i][-32:-16], got[32:]) == \
            jobs[k]["cookie"].tobytes()


def test_mac2_check_rejects_non_handshake_lengths(torch_cuda, gpu):
    """Only 148- and 92-byte messages reach the mac2 check (parse_incoming_packet,
    noise/mod.rs:139-199); any other length -- 0, 16 (len - 16 would wrap), 91,
    147, 200 (past the slot) -- gets WG_STATUS_INVALID_PACKET and a zero cookie,
    without the kernel reading the message, while valid neighbours still check."""
    torch = torch_cuda
    from neptun_amd import gpu as G
    rng = random.Random(41)
    secret = rng.randbytes(16)
    counter = rng.getrandbits(40)
    lens = [0, 16, 148, 91, 147, 200, 92, 0xFFFFFFF0]
    n = len(lens)
    stride = 148
    d_m = to_dev(torch, rng.randbytes(stride * n))
    d_l = to_dev(torch, np.array(lens, np.uint32).tobytes())
    addrs = [rng.randbytes(16) for _ in range(n)]
    d_a = to_dev(torch, b"".join(addrs))
    d_c = torch.full((16 * n,), 0xAB, dtype=torch.uint8, device="cuda")
    d_st = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    gpu.mac2_check_batch(secret, counter, n, d_m, stride, d_l, d_a, d_c, d_st)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    cookies = d_c.cpu().numpy().tobytes()
    for i, ln in enumerate(lens):
        if ln in (148, 92):
            assert st[i] in (0, 1)
            assert cookies[16 * i:16 * i + 16] == H.current_cookie(secret, counter, addrs[i])
        else:
            assert G.STATUS[int(st[i])] == "InvalidPacket", (i, ln)
            assert cookies[16 * i:16 * i + 16] == bytes(16)


def test_initiator_handshake_on_gpu_end_to_end(torch_cuda, gpu):
    """Initiator side: format_handshake_initiation + mac1/mac2
    (handshake.rs:769-851, :732-765) on the device equals the oracle's initiation
    (message, InitSent chaining key / hash, last mac1); the device responder
    (consume + respond) answers; receive_handshake_response (:615-695) on the
    device equals the oracle's receive_response and yields the responder's keys
    crossed (initiator sending = responder receiving = temp2).  Damaged responses
    fail as the reference fails them: InvalidMac (mac1 checked), InvalidAeadTag
    (mac1 not checked), WrongPacketType."""
    from neptun_amd import gpu as G
    torch = torch_cuda
    rng = random.Random(61)
    resp_priv = rng.randbytes(32)
    resp_pub = H.public_key(resp_priv)
    n = 260
    jobs = np.zeros(n, G.INITIATION_JOB_DTYPE)
    want = []
    for i in range(n):
        si, ei, ts = rng.randbytes(32), rng.randbytes(32), rng.randbytes(12)
        cookie = rng.randbytes(16) if i % 3 == 0 else None
        idx = rng.getrandbits(32)
        jobs[i]["ephemeral_private"] = np.frombuffer(ei, np.uint8)
        jobs[i]["static_public"] = np.frombuffer(H.public_key(si), np.uint8)
        jobs[i]["peer_static_public"] = np.frombuffer(resp_pub, np.uint8)
        jobs[i]["static_shared"] = np.frombuffer(H.x25519(si, resp_pub), np.uint8)
        jobs[i]["mac1_key"] = np.frombuffer(H.b2s_hash(H.LABEL_MAC1, resp_pub), np.uint8)
        jobs[i]["timestamp"] = np.frombuffer(ts, np.uint8)
        jobs[i]["local_index"] = idx
        jobs[i]["has_cookie"] = 1 if cookie else 0
        jobs[i]["cookie"] = np.frombuffer(cookie or bytes(16), np.uint8)
        want.append((si, ei, idx) + H.initiation(si, resp_pub, ei, idx, ts, cookie))
    d_j = to_dev(torch, jobs.tobytes())
    d_o = torch.zeros(n * G.INIT_SENT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    gpu.handshake_initiate_batch(n, d_j, d_o)
    torch.cuda.synchronize()
    sent = d_o.cpu().numpy().view(G.INIT_SENT_DTYPE)
    for i, (si, ei, idx, msg, ck, h) in enumerate(want):
        assert sent[i]["message"].tobytes() == msg, i
        assert int(sent[i]["local_index"]) == idx
        assert sent[i]["chaining_key"].tobytes() == ck and sent[i]["hash"].tobytes() == h
        assert sent[i]["mac1"].tobytes() == msg[116:132]
    # the device responder answers the device initiations
    msgs = b"".join(sent[i]["message"].tobytes() for i in range(n))
    peers = np.zeros(n, G.RESPONDER_PEER_DTYPE)
    for i, (si, *_rest) in enumerate(want):
        pi = H.public_key(si)
        peers[i]["peer_static_public"] = np.frombuffer(pi, np.uint8)
        peers[i]["static_shared"] = np.frombuffer(H.x25519(resp_priv, pi), np.uint8)
    d_s = torch.zeros(n * G.INIT_RECEIVED_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    gpu.handshake_consume_batch(resp_priv, n, to_dev(torch, msgs), 148, to_dev(torch, peers.tobytes()), d_s)
    rjobs = np.zeros(n, G.RESPONSE_JOB_DTYPE)
    psks = []
    for i, (si, *_rest) in enumerate(want):
        psk = rng.randbytes(32) if i % 4 == 1 else bytes(32)
        psks.append(psk)
        rjobs[i]["ephemeral_private"] = np.frombuffer(rng.randbytes(32), np.uint8)
        rjobs[i]["peer_static_public"] = peers[i]["peer_static_public"]
        rjobs[i]["preshared_key"] = np.frombuffer(psk, np.uint8)
        rjobs[i]["mac1_key"] = np.frombuffer(H.b2s_hash(H.LABEL_MAC1, H.public_key(si)), np.uint8)
        rjobs[i]["local_index"] = 0x0A000000 + i
    d_r = torch.zeros(n * G.RESPONSE_OUT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    gpu.handshake_respond_batch(n, d_s, to_dev(torch, rjobs.tobytes()), d_r)
    torch.cuda.synchronize()
    resp = d_r.cpu().numpy().view(G.RESPONSE_OUT_DTYPE)
    assert (d_s.cpu().numpy().view(G.INIT_RECEIVED_DTYPE)["status"] == 0).all()
    # damage some responses: mac1-checked batch sees InvalidMac, unchecked InvalidAeadTag
    rmsgs, kind = [], []
    for i in range(n):
        m = bytearray(resp[i]["message"].tobytes())
        r = i % 10
        if r == 7:
            m[rng.randrange(44, 60)] ^= 0x20   # encrypted nothing (its tag)
            kind.append("tag")
        elif r == 8:
            m[0] = 1
            kind.append("type")
        else:
            kind.append("ok")
        rmsgs.append(bytes(m))
    stride = 96
    d_m = to_dev(torch, b"".join(m + bytes(stride - 92) for m in rmsgs))
    ijobs = np.zeros(n, G.RESPONSE_RECEIVED_JOB_DTYPE)
    for i, (si, ei, idx, msg, ck, h) in enumerate(want):
        ijobs[i]["chaining_key"] = np.frombuffer(ck, np.uint8)
        ijobs[i]["hash"] = np.frombuffer(h, np.uint8)
        ijobs[i]["ephemeral_private"] = np.frombuffer(ei, np.uint8)
        ijobs[i]["preshared_key"] = np.frombuffer(psks[i], np.uint8)
    d_ij = to_dev(torch, ijobs.tobytes())
    for check_mac1 in (True, False):
        out = torch.zeros(n * G.SESSION_KEYS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        res = np.zeros(n, G.SESSION_KEYS_DTYPE)
        # the initiator's static key is one per call (wave-uniform) and every
        # initiation above has its own: one single-entry call each for a sample,
        # plus one whole-batch call with the first initiator's key below
        for i in range(0, n, 13):
            si = want[i][0]
            o1 = torch.zeros(G.SESSION_KEYS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
            gpu.handshake_receive_response_batch(si, 1, d_m[stride * i:], stride,
                                                 d_ij[G.RESPONSE_RECEIVED_JOB_DTYPE.itemsize * i:], o1,
                                                 check_mac1=check_mac1)
            torch.cuda.synchronize()
            res[i] = o1.cpu().numpy().view(G.SESSION_KEYS_DTYPE)[0]
        for i in range(0, n, 13):
            si, ei, idx, msg, ck, h = want[i]
            st = int(res[i]["status"])
            if kind[i] == "type":
                assert st == H.WRONG_PACKET_TYPE, i
                continue
            if kind[i] == "tag":
                assert st == (H.INVALID_MAC if check_mac1 else H.INVALID_AEAD_TAG), (i, st)
                continue
            exp = H.receive_response(ck, h, ei, si, rmsgs[i], psks[i])
            assert st == exp[0] == 0, (i, st)
            assert int(res[i]["peer_index"]) == 0x0A000000 + i
            assert int(res[i]["receiver_idx"]) == idx  # the initiator's local index: picks the state
            assert res[i]["sending_key"].tobytes() == exp[1] == resp[i]["receiving_key"].tobytes()
            assert res[i]["receiving_key"].tobytes() == exp[2] == resp[i]["sending_key"].tobytes()
        # whole batch under initiator 0's key: only entry 0 (and any other entry of
        # that key) derives the right keys; the rest fail their AEAD tag
        gpu.handshake_receive_response_batch(want[0][0], n, d_m, stride, d_ij, out, check_mac1=False)
        torch.cuda.synchronize()
        allres = out.cpu().numpy().view(G.SESSION_KEYS_DTYPE)
        assert int(allres[0]["status"]) == 0
        assert all(int(allres[i]["status"]) in (H.INVALID_AEAD_TAG, H.WRONG_PACKET_TYPE) for i in range(1, n))
        # a job that is not the InitSent state of the message's receiver index (states
        # swapped): InvalidAeadTag, and receiver_idx names the state the caller should
        # have picked
        ok_i = [i for i in range(n) if kind[i] == "ok"][:2]
        a, b = ok_i
        o1 = torch.zeros(G.SESSION_KEYS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        gpu.handshake_receive_response_batch(want[a][0], 1, d_m[stride * a:], stride,
                                             d_ij[G.RESPONSE_RECEIVED_JOB_DTYPE.itemsize * b:], o1,
                                             check_mac1=check_mac1)
        torch.cuda.synchronize()
        r1 = o1.cpu().numpy().view(G.SESSION_KEYS_DTYPE)[0]
        assert int(r1["status"]) == H.INVALID_AEAD_TAG and int(r1["receiver_idx"]) == want[a][2]


def test_cookie_reply_open_matches_oracle(torch_cuda, gpu):
    """receive_cookie_reply (handshake.rs:697-727): the device responder's COOKIE_REPLY
    messages (cookie_reply_batch) opened on the device give back the cookies;
    a damaged tag or ciphertext -> InvalidAeadTag (cookie zeroed), a wrong type ->
    WrongPacketType; the receiver index comes back for the caller's cookies.index check."""
    from neptun_amd import gpu as G
    torch = torch_cuda
    rng = random.Random(67)
    resp_pub = H.public_key(rng.randbytes(32))
    cookie_key = H.b2s_hash(H.LABEL_COOKIE, resp_pub)
    nonce_key = rng.randbytes(32)
    n = 300
    rj = np.zeros(n, G.COOKIE_REPLY_JOB_DTYPE)
    for i in range(n):
        rj[i]["cookie"] = np.frombuffer(rng.randbytes(16), np.uint8)
        rj[i]["mac1"] = np.frombuffer(rng.randbytes(16), np.uint8)
        rj[i]["nonce_ctr"] = 1000 + i
        rj[i]["receiver_idx"] = rng.getrandbits(32)
    d_o = torch.zeros(64 * n, dtype=torch.uint8, device="cuda")
    gpu.cookie_reply_batch(cookie_key, nonce_key, n, to_dev(torch, rj.tobytes()), d_o)
    torch.cuda.synchronize()
    replies = d_o.cpu().numpy().tobytes()
    oj = np.zeros(n, G.COOKIE_OPEN_JOB_DTYPE)
    kinds = []
    for i in range(n):
        m = bytearray(replies[64 * i:64 * i + 64])
        assert bytes(m) == H.format_cookie_reply(cookie_key, int(rj[i]["receiver_idx"]), rj[i]["cookie"].tobytes(),
                                                 rj[i]["mac1"].tobytes(), H.cookie_nonce(nonce_key, 1000 + i))
        k = i % 8
        if k == 5:
            m[rng.randrange(32, 64)] ^= 4
        elif k == 6:
            m[0] = 2
        kinds.append(k)
        oj[i]["message"] = np.frombuffer(bytes(m), np.uint8)
        oj[i]["cookie_key"] = np.frombuffer(cookie_key, np.uint8)
        mac1 = rj[i]["mac1"].tobytes() if k != 7 else rng.randbytes(16)  # wrong AAD
        oj[i]["mac1"] = np.frombuffer(mac1, np.uint8)
    d_res = torch.zeros(n * G.COOKIE_OPEN_OUT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    gpu.cookie_reply_open_batch(n, to_dev(torch, oj.tobytes()), d_res)
    torch.cuda.synchronize()
    res = d_res.cpu().numpy().view(G.COOKIE_OPEN_OUT_DTYPE)
    for i in range(n):
        st, k = int(res[i]["status"]), kinds[i]
        assert int(res[i]["receiver_idx"]) == (int(rj[i]["receiver_idx"]) if k != 6 else
                                                int.from_bytes(oj[i]["message"][4:8].tobytes(), "little"))
        if k == 6:
            assert st == H.WRONG_PACKET_TYPE
        elif k in (5, 7):
            assert st == H.INVALID_AEAD_TAG and res[i]["cookie"].tobytes() == bytes(16), i
        else:
            m = oj[i]["message"].tobytes()
            want = H.xchacha20poly1305_open(cookie_key, m[8:32], rj[i]["mac1"].tobytes(), m[32:])
            assert st == 0 and res[i]["cookie"].tobytes() == want == rj[i]["cookie"].tobytes(), i
