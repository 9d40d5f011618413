#!/usr/bin/env python3
"""Throughput of the batched handshake kernels, one JSON line each:
X25519 operations per second (per-lane scalar and point), handshake initiations
per second through mac1 + parse_handshake_anon, the responder's consume / respond,
the cookie path and the initiator's initiate / receive-response, next to OpenSSL's X25519 on the host
cores (oracle/build/cpu_x25519, 16 threads; the reference's x25519-dalek cannot be
built here).  Inputs are device-resident; every output of the timed run is checked
on a sample against oracle/handshake_model.py."""
import json
import os
import random
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import neptun_amd
    from neptun_amd.gpu import HALF_HANDSHAKE_DTYPE
    from oracle import handshake_model as H
    n = int(os.environ.get("HS_N", 1 << 20))
    ctx = neptun_amd.GpuContext(0, key_slots=1)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    sc = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device="cuda", generator=g)
    pt = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ctx.x25519_batch(n, sc, pt, out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record()
        ctx.x25519_batch(n, sc, pt, out)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    s, p, o = sc.cpu().numpy().tobytes(), pt.cpu().numpy().tobytes(), out.cpu().numpy().tobytes()
    rng = random.Random(2)
    ok = all(o[32 * i:32 * i + 32] == H.x25519(s[32 * i:32 * i + 32], p[32 * i:32 * i + 32])
             for i in rng.sample(range(n), 64))
    t = statistics.median(ts)
    print(json.dumps({"op": "x25519", "n": n, "ms": round(t * 1e3, 3),
                      "ops_per_s": round(n / t, 1), "verified_sample": ok}), flush=True)

    # handshake initiations: 4096 distinct valid messages tiled over the batch
    resp_priv = bytes(range(32))
    resp_pub = H.public_key(resp_priv)
    init_privs = [rng.randbytes(32) for _ in range(512)]
    base = [H.format_handshake_initiation(init_privs[i], resp_pub, rng.randbytes(32), i,
                                          rng.randbytes(12)) for i in range(512)]
    tile = b"".join(base)
    msgs = torch.from_numpy(np.frombuffer(tile * (n // len(base)), np.uint8).copy()).cuda()
    m = n // len(base) * len(base)
    res = torch.zeros(m * HALF_HANDSHAKE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ctx.handshake_anon_batch(resp_priv, m, msgs, 148, res)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record()
        ctx.handshake_anon_batch(resp_priv, m, msgs, 148, res)
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    r = res.cpu().numpy().view(HALF_HANDSHAKE_DTYPE)
    ok = bool((r["status"] == 0).all()) and all(
        r[i]["peer_static_public"].tobytes() ==
        H.parse_handshake_anon(resp_priv, resp_pub, base[i % len(base)])[2]
        for i in rng.sample(range(m), 32))
    t = statistics.median(ts)
    print(json.dumps({"op": "handshake_anon (mac1 + parse_handshake_anon)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)

    # responder: receive_handshake_initialization crypto, then format_handshake_response
    from neptun_amd import gpu as G

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        tt = []
        for _ in range(5):
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            tt.append(ev[0].elapsed_time(ev[1]) * 1e-3)
        return statistics.median(tt)

    peers_base = np.zeros(len(base), G.RESPONDER_PEER_DTYPE)
    for i, k in enumerate(init_privs):
        pub = H.public_key(k)
        peers_base[i]["peer_static_public"] = np.frombuffer(pub, np.uint8)
        peers_base[i]["static_shared"] = np.frombuffer(H.x25519(resp_priv, pub), np.uint8)
    peers = torch.from_numpy(np.tile(peers_base, m // len(base)).view(np.uint8).copy()).cuda()
    states = torch.zeros(m * G.INIT_RECEIVED_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    t = timed(lambda: ctx.handshake_consume_batch(resp_priv, m, msgs, 148, peers, states))
    st = states.cpu().numpy().view(G.INIT_RECEIVED_DTYPE)
    ok = bool((st["status"] == 0).all())
    for i in rng.sample(range(m), 16):
        want = H.consume_initiation(resp_priv, peers_base[i % len(base)]["peer_static_public"].tobytes(),
                                    peers_base[i % len(base)]["static_shared"].tobytes(),
                                    base[i % len(base)])
        ok = ok and st[i]["chaining_key"].tobytes() == want[3] and st[i]["hash"].tobytes() == want[4]
    print(json.dumps({"op": "handshake_consume (receive_handshake_initialization crypto)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)
    jobs_np = np.zeros(m, G.RESPONSE_JOB_DTYPE)
    jobs_np["ephemeral_private"] = np.frombuffer(rng.randbytes(32 * m), np.uint8).reshape(m, 32)
    jobs_np["peer_static_public"] = np.tile(peers_base, m // len(base))["peer_static_public"]
    # the response's mac1 is keyed by the INITIATOR's static public key
    mac1_keys = np.stack([np.frombuffer(H.b2s_hash(H.LABEL_MAC1, p["peer_static_public"].tobytes()),
                                        np.uint8) for p in peers_base])
    jobs_np["mac1_key"] = np.tile(mac1_keys, (m // len(base), 1))
    jobs_np["local_index"] = np.arange(m, dtype=np.uint32)
    jobs = torch.from_numpy(jobs_np.view(np.uint8).copy()).cuda()
    outs = torch.zeros(m * G.RESPONSE_OUT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    t = timed(lambda: ctx.handshake_respond_batch(m, states, jobs, outs))
    o = outs.cpu().numpy().view(G.RESPONSE_OUT_DTYPE)
    ok = True
    for i in rng.sample(range(m), 8):
        _, idx, ts_, ck, h, eph = H.consume_initiation(
            resp_priv, peers_base[i % len(base)]["peer_static_public"].tobytes(),
            peers_base[i % len(base)]["static_shared"].tobytes(), base[i % len(base)])
        resp = H.format_response(ck, h, eph, idx, i, jobs_np[i]["ephemeral_private"].tobytes(),
                                 jobs_np[i]["peer_static_public"].tobytes())[0]
        ok = ok and o[i]["message"].tobytes() == resp
    print(json.dumps({"op": "handshake_respond (format_handshake_response + mac1)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)
    # under load: mac2 check of every initiation, cookie reply for each
    lens = torch.full((m,), 148, dtype=torch.int32, device="cuda")
    addrs = torch.randint(0, 256, (16 * m,), dtype=torch.uint8, device="cuda", generator=g)
    cookies = torch.zeros(16 * m, dtype=torch.uint8, device="cuda")
    cst = torch.zeros(m, dtype=torch.int32, device="cuda")
    secret = rng.randbytes(16)
    t = timed(lambda: ctx.mac2_check_batch(secret, 7, m, msgs, 148, lens, addrs, cookies, cst))
    ok = bool((cst == 1).all())
    print(json.dumps({"op": "mac2_check (current_cookie + mac2, under load)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)
    cj = np.zeros(m, G.COOKIE_REPLY_JOB_DTYPE)
    cj["cookie"] = cookies.cpu().numpy().reshape(m, 16)
    cj["nonce_ctr"] = np.arange(m, dtype=np.uint64)
    d_cj = torch.from_numpy(cj.view(np.uint8).copy()).cuda()
    replies = torch.zeros(64 * m, dtype=torch.uint8, device="cuda")
    ck_key, n_key = H.b2s_hash(H.LABEL_COOKIE, resp_pub), rng.randbytes(32)
    t = timed(lambda: ctx.cookie_reply_batch(ck_key, n_key, m, d_cj, replies))
    rb = replies.cpu().numpy().tobytes()
    ok = all(rb[64 * i:64 * i + 64] == H.format_cookie_reply(ck_key, 0, cj[i]["cookie"].tobytes(),
                                                            bytes(16), H.cookie_nonce(n_key, i))
             for i in rng.sample(range(m), 16))
    print(json.dumps({"op": "cookie_reply (XChaCha20-Poly1305)", "n": m, "ms": round(t * 1e3, 3),
                      "msgs_per_s": round(m / t, 1), "verified_sample": ok}), flush=True)
    # initiator side: format_handshake_initiation for m peers, then receive_handshake_response
    # of the device responder's answers (one local static key, as on one interface)
    init_priv = rng.randbytes(32)
    init_pub = H.public_key(init_priv)
    peer_privs = [rng.randbytes(32) for _ in range(len(base))]
    peer_pubs = [H.public_key(k) for k in peer_privs]
    ij = np.zeros(m, G.INITIATION_JOB_DTYPE)
    ij["ephemeral_private"] = np.frombuffer(rng.randbytes(32 * m), np.uint8).reshape(m, 32)
    ij["static_public"] = np.frombuffer(init_pub, np.uint8)
    pp = np.stack([np.frombuffer(x, np.uint8) for x in peer_pubs])
    ss = np.stack([np.frombuffer(H.x25519(init_priv, x), np.uint8) for x in peer_pubs])
    mk = np.stack([np.frombuffer(H.b2s_hash(H.LABEL_MAC1, x), np.uint8) for x in peer_pubs])
    reps = m // len(base)
    ij["peer_static_public"] = np.tile(pp, (reps, 1))
    ij["static_shared"] = np.tile(ss, (reps, 1))
    ij["mac1_key"] = np.tile(mk, (reps, 1))
    ij["timestamp"] = np.frombuffer(rng.randbytes(12), np.uint8)
    ij["local_index"] = np.arange(m, dtype=np.uint32)
    d_ij = torch.from_numpy(ij.view(np.uint8).copy()).cuda()
    sent = torch.zeros(m * G.INIT_SENT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    t = timed(lambda: ctx.handshake_initiate_batch(m, d_ij, sent))
    sn = sent.cpu().numpy().view(G.INIT_SENT_DTYPE)
    ok = True
    for i in rng.sample(range(m), 8):
        want = H.initiation(init_priv, peer_pubs[i % len(base)], ij[i]["ephemeral_private"].tobytes(), i,
                            ij[i]["timestamp"].tobytes())
        ok = ok and sn[i]["message"].tobytes() == want[0] and sn[i]["hash"].tobytes() == want[2]
    print(json.dumps({"op": "handshake_initiate (format_handshake_initiation + mac1)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)
    # responses to time receive_response on: the oracle answers a tile, repeated (the
    # kernel's work does not depend on which response it opens)
    tile_r, rj_tile = [], np.zeros(len(base), G.RESPONSE_RECEIVED_JOB_DTYPE)
    for i in range(len(base)):
        _, idx, _ts, ck, h, eph = H.consume_initiation(peer_privs[i], init_pub, H.x25519(peer_privs[i], init_pub),
                                                        sn[i]["message"].tobytes())
        tile_r.append(H.format_response(ck, h, eph, idx, 7 + i, rng.randbytes(32), init_pub)[0])
        rj_tile[i]["chaining_key"] = sn[i]["chaining_key"]
        rj_tile[i]["hash"] = sn[i]["hash"]
        rj_tile[i]["ephemeral_private"] = ij[i]["ephemeral_private"]
    d_rm = torch.from_numpy(np.frombuffer(b"".join(tile_r) * reps, np.uint8).copy()).cuda()
    d_rj = torch.from_numpy(np.tile(rj_tile, reps).view(np.uint8).copy()).cuda()
    keys_out = torch.zeros(m * G.SESSION_KEYS_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    t = timed(lambda: ctx.handshake_receive_response_batch(init_priv, m, d_rm, 92, d_rj, keys_out))
    ko = keys_out.cpu().numpy().view(G.SESSION_KEYS_DTYPE)
    ok = bool((ko["status"] == 0).all())
    for i in rng.sample(range(m), 8):
        j = i % len(base)
        want = H.receive_response(sn[j]["chaining_key"].tobytes(), sn[j]["hash"].tobytes(),
                                  ij[j]["ephemeral_private"].tobytes(), init_priv, tile_r[j])
        ok = ok and ko[i]["sending_key"].tobytes() == want[1]
    print(json.dumps({"op": "handshake_receive_response (mac1 + receive_handshake_response)", "n": m,
                      "ms": round(t * 1e3, 3), "msgs_per_s": round(m / t, 1),
                      "verified_sample": ok}), flush=True)
    exe = os.path.join(ROOT, "oracle", "build", "cpu_x25519")
    if os.path.exists(exe):
        threads = min(16, len(os.sched_getaffinity(0)))
        for th in (1, threads):
            r = subprocess.run([exe, "--threads", str(th), "--ops", "20000"], capture_output=True,
                               text=True, timeout=300)
            print(json.dumps({"op": "cpu_baseline x25519 (OpenSSL 3 EVP)", **json.loads(r.stdout)}),
                  flush=True)


if __name__ == "__main__":
    main()
