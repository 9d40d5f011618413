#!/usr/bin/env python3
"""Randomized soak of the product kernels on one GPU (rare-race / hazard hunt).

For SECONDS seconds: pick a random batch shape, seal it twice -- through the
strided API (uniform kernels) and through the descriptor API (the descriptor
forms the host picks for that launch) -- and require the two destination
buffers, canaries included, to be byte-identical; open both back and require
the plaintext, statuses and untouched canaries; every few iterations also a
mixed-length descriptor batch through the plan (ordered launch) against its
unordered twin, and every third a batch with a random key slot per packet (a
4096-slot table: the affine descriptor kernel against the plan-ordered one).  The
unordered descriptor launch draws its form at random (round 5): the throughput kernels,
the default selection, or the latency form with a forced group of 2 .. 64 lanes per
packet (wg_xlane.hip) -- and so does the descriptor open.  Round 6: long packets (up to
8192 B) too, and the strided seal draws its split (wg_gpu_ctx_set_split: the default
choice, unsplit, or K = 2 ... 8 parts per wave with the finish kernel).  A one-in-a-million
corruption in any form shows up as a mismatch between forms that share no kernel.
Prints one JSON summary line.

    python tools/stress.py [SECONDS] [OUT.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import neptun_amd
    from oracle import pyoracle as o
    from tools import synth
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(int(time.time()) & 0xFFFF)
    seed = int(rng.integers(1 << 30))
    ctx1 = neptun_amd.GpuContext(0, key_slots=1)
    ctx1.set_keys(0, synth.keys(1, seed=seed), np.array([synth.RECEIVER_IDX], np.uint32))
    # per-packet keys (config 4's shape): a 4096-slot table, random slot per packet
    ctxk = neptun_amd.GpuContext(0, key_slots=4096)
    ctxk.set_keys(0, synth.keys(4096, seed=seed + 1),
                  np.full(4096, synth.RECEIVER_IDX, np.uint32) + np.arange(4096, dtype=np.uint32))
    ctx1.set_xlane_lanes(0)
    ctxk.set_xlane_lanes(0)
    stats = {"seed": seed, "iterations": 0, "packets": 0, "bytes": 0, "mismatches": [], "forms": {}}
    t_end = time.time() + seconds
    last_print = time.time()
    it = 0
    while time.time() < t_end:
        it += 1
        mixed = it % 5 == 0
        keyed = it % 3 == 0 and not mixed  # per-packet keys: two descriptor forms, no strided one
        ctx = ctxk if keyed else ctx1
        n = int(rng.choice([64, 4096, 65536, 262144, 1 << 20])) + int(rng.integers(0, 64))
        if mixed:
            n = min(n, 200000)
            sizes = rng.choice([0, 64, 256, 576, 1350, 1500, 8900], n)
            S = 9088
        else:
            P = int(rng.choice([64, 576, 1350, 1420, int(rng.integers(0, 2000)), 4096, 8192,
                                int(rng.integers(2000, 9000))]))
            if P > 2000:
                n = min(n, 262144 + int(rng.integers(0, 64)))
            sizes = np.full(n, P, np.int64)
            S = synth.round_up(P + 32 + int(rng.choice([0, 16, 96])), 16)
        sizes_t = torch.from_numpy(sizes.astype(np.int64)).to(dev)
        pt = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device=dev)
        ctr0 = int(rng.integers(0, 2**40))
        descs = np.zeros(n, o.DESC_DTYPE)
        descs["src_off"] = np.arange(n, dtype=np.int64) * S
        descs["dst_off"] = np.arange(n, dtype=np.int64) * S
        descs["counter"] = ctr0 + np.arange(n, dtype=np.uint64)
        descs["len"] = sizes
        if keyed:
            descs["key_slot"] = rng.integers(0, 4096, n).astype(np.uint32)
        d_descs = torch.from_numpy(descs.view(np.uint8)).to(dev)
        outs, sts = [], []
        forms = ["desc-ordered", "desc"] if (mixed or keyed) else ["strided", "desc"]

        def pick_xlane():  # the unordered descriptor launch's form
            c = int(rng.integers(0, 4))
            if c == 0:
                ctx.set_xlane_lanes(0)
                return "tput"
            if c == 1:
                ctx.set_xlane_lanes(-1)
                return "default"
            G = int(rng.choice([2, 4, 8, 16, 32, 64]))
            ctx.set_xlane_lanes(n * G)
            return f"xlane{G}"
        for form in forms:
            w = torch.full((n * S + 64,), 0xA5, dtype=torch.uint8, device=dev)
            st = torch.full((n,), -1, dtype=torch.int32, device=dev)
            if form == "strided":
                K = int(rng.choice([-1, 1, 2, 3, 4, 5, 6, 7, 8]))
                ctx.set_split(K)
                form = f"strided-split{K}"
                ctx.seal_strided(n, int(sizes[0]), 0, ctr0, pt, S, w, S, st)
                ctx.set_split(-1)
            elif form == "desc-ordered":
                order = torch.zeros(n, dtype=torch.int32, device=dev)
                scratch = torch.zeros(262144 // 4, dtype=torch.int32, device=dev)
                ctx.plan_batch(True, d_descs, n, order, scratch)
                ctx.seal_batch_ordered(d_descs, order, n, pt, w, st)
            else:
                form = form + "-" + pick_xlane()
                ctx.seal_batch(d_descs, n, pt, w, st)
                ctx.set_xlane_lanes(0)  # (the ordered launches: the throughput kernels)
            outs.append(w)
            sts.append(st)
            tag = form + ("-keyed" if keyed else "")
            stats["forms"][tag] = stats["forms"].get(tag, 0) + 1
        torch.cuda.synchronize()
        bad = []
        if not torch.equal(outs[0], outs[1]):
            diff = torch.nonzero(outs[0] != outs[1]).flatten()
            bad.append({"what": "seal forms differ", "first_byte": int(diff[0]), "bytes": int(diff.numel())})
        if int((sts[0] != 0).sum()) or int((sts[1] != 0).sum()):
            bad.append({"what": "seal status"})
        # open the first form's datagrams back (descriptor API; the strided one on uniform batches)
        d2 = descs.copy()
        d2["len"] = sizes + 32
        back = torch.full((n * S + 64,), 0x5A, dtype=torch.uint8, device=dev)
        st2 = torch.full((n,), -1, dtype=torch.int32, device=dev)
        if mixed or keyed or it % 2 == 0:
            tag = "open-" + pick_xlane()
            stats["forms"][tag] = stats["forms"].get(tag, 0) + 1
            ctx.open_batch(torch.from_numpy(d2.view(np.uint8)).to(dev), n, outs[0], back, st2)
            ctx.set_xlane_lanes(0)
        else:
            K = int(rng.choice([-1, 1, 2, 3, 4, 5, 6, 7, 8]))
            ctx.set_split(K)
            tag = f"open-strided-split{K}"
            stats["forms"][tag] = stats["forms"].get(tag, 0) + 1
            ctx.open_strided(n, int(sizes[0]) + 32, 0, outs[0], S, back, S, st2)
            ctx.set_split(-1)
        torch.cuda.synchronize()
        if int((st2 != 0).sum()):
            bad.append({"what": "open status", "failed": int((st2 != 0).sum())})
        # plaintext back in every slot's first len bytes, canary everywhere else
        idx = torch.arange(S, device=dev).view(1, S)
        inside = idx < sizes_t.view(n, 1)
        bv, pv = back[: n * S].view(n, S), pt.view(n, S)
        if not torch.equal(torch.where(inside, bv, torch.full_like(bv, 0x5A)), torch.where(inside, pv, torch.full_like(pv, 0x5A))) \
                or int((back[n * S:] != 0x5A).sum()):
            bad.append({"what": "open bytes"})
        stats["iterations"] += 1
        stats["packets"] += 2 * n
        if time.time() - last_print > 30:  # progress (a long soak must not look hung)
            last_print = time.time()
            print(json.dumps({"progress_s": round(seconds - (t_end - last_print), 1),
                              "iterations": stats["iterations"], "packets": stats["packets"],
                              "mismatches": len(stats["mismatches"])}), flush=True)
        stats["bytes"] += 2 * int(sizes.sum())
        if bad:
            stats["mismatches"].append({"iteration": it, "n": n, "mixed": mixed, "keyed": keyed, "stride": S,
                                        "problems": bad})
            if len(stats["mismatches"]) > 5:
                break
        del pt, outs, back
    stats["seconds"] = seconds
    stats["ok"] = not stats["mismatches"]
    print(json.dumps(stats), flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump(stats, f, indent=1)
    sys.exit(0 if stats["ok"] else 1)


if __name__ == "__main__":
    main()
