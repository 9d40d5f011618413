#!/usr/bin/env python3
"""Debug helper: run seal/open of two builds of libneptun_gpu.so on the same
1M x 1350 B batch and report where their outputs differ (packet index, lane,
wave, byte range).

    python tools/diff_variants.py build/variants/libneptun_gpu_ref.so build/variants/libneptun_gpu_new.so
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.ab import bind  # noqa: E402


def main():
    import torch
    from tools import synth
    n, P = 1 << 20, int(os.environ.get("DIFF_SIZE", 1350))
    S = synth.round_up(P + 32, 128)
    off = int(os.environ.get("DIFF_OFFSET", 16))
    dev = torch.device("cuda", 0)
    pt = synth.device_payloads(n, P, S, dev, offset=off)
    key = synth.keys(1)
    idx = np.array([synth.RECEIVER_IDX], np.uint32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    libs = []
    for p in sys.argv[1:3]:
        L = bind(p)
        h = ctypes.c_void_p()
        assert L.wg_gpu_ctx_create(0, 1, ctypes.byref(h)) == 0
        assert L.wg_gpu_set_keys(h, 0, 1, key.ctypes.data, idx.ctypes.data, stream) == 0
        libs.append((L, h))
    for L, h in libs:
        wire = torch.zeros(n * S, dtype=torch.uint8, device=dev)
        st = torch.full((n,), -1, dtype=torch.int32, device=dev)
        assert L.wg_gpu_seal_strided(h, n, P, 0, 0, pt.data_ptr() + off, S, wire.data_ptr(), S, st.data_ptr(), stream) == 0
        torch.cuda.synchronize()
        outs.append((wire, st.clone()))
    (wa, sa), (wb, sb) = outs
    d = (wa.view(n, S)[:, :P + 32] != wb.view(n, S)[:, :P + 32])
    bad = torch.nonzero(d.any(dim=1)).flatten().cpu().numpy()
    print(f"seal: {len(bad)} packets differ; status nonzero ref {int((sa != 0).sum())} new {int((sb != 0).sum())}")
    if len(bad):
        print("  first packets:", bad[:20].tolist())
        print("  lanes:", np.bincount(bad % 64, minlength=64).tolist())
        print("  wave-in-group (8/wg):", np.bincount((bad // 64) % 8, minlength=8).tolist())
        cols = torch.nonzero(d[torch.from_numpy(bad[:2000]).to(dev)].any(dim=0)).flatten().cpu().numpy()
        print("  differing byte columns (wire offset) min/max:", cols.min(), cols.max(), "rounds:", sorted(set((cols // 128).tolist())))
        g = bad // 512
        print("  groups (512 pkts):", len(set(g.tolist())), "first:", sorted(set(g.tolist()))[:20])
    # open the reference wire with both
    for name, (L, h) in zip(("ref", "new"), libs):
        back = torch.zeros(n * S, dtype=torch.uint8, device=dev)
        st = torch.full((n,), -1, dtype=torch.int32, device=dev)
        assert L.wg_gpu_open_strided(h, n, P + 32, 0, wa.data_ptr(), S, back.data_ptr() + off, S, st.data_ptr(), stream) == 0
        torch.cuda.synchronize()
        badst = torch.nonzero(st != 0).flatten().cpu().numpy()
        dd = (back.view(n, S)[:, off:off + P] != pt.view(n, S)[:, off:off + P]).any(dim=1)
        badpt = torch.nonzero(dd).flatten().cpu().numpy()
        print(f"open[{name}] of ref wire: {len(badst)} bad status, {len(badpt)} bad plaintext; first {badst[:10].tolist()}")


if __name__ == "__main__":
    main()
