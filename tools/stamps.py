#!/usr/bin/env python3
"""Phase timing of the phase-locked strided kernel from in-kernel s_memtime
stamps (diagnostic build: make -C neptun_amd/csrc variant NAME=stamp DEFS=-DWG_STAMP=1).

    python tools/stamps.py build/variants/libneptun_gpu_stamp.so

Phases per round (wave 0 of each workgroup): 0 round start, 1 DMA issued,
2 keystream done, 3 DMA landed, 4 XOR+Poly done, 5 stores issued.  Prints the
median cycles of each phase over workgroups for every round.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.ab import bind  # noqa: E402

BLOCKS, ROUNDS, PHASES = 4096, 16, 6
NAMES = ["issue DMA", "keystream", "wait DMA", "xor+poly", "stores", "-> next round"]


def main():
    import torch
    from tools import synth
    L = bind(sys.argv[1])
    L.wg_gpu_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    n, P = 1 << 20, 1350
    S = synth.round_up(P + 32, 128)
    dev = torch.device("cuda", 0)
    pt = synth.device_payloads(n, P, S, dev, offset=16)
    wire = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    back = torch.zeros(n * S, dtype=torch.uint8, device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    key = synth.keys(1)
    idx = np.array([synth.RECEIVER_IDX], np.uint32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    h = ctypes.c_void_p()
    assert L.wg_gpu_ctx_create(0, 1, ctypes.byref(h)) == 0
    assert L.wg_gpu_set_keys(h, 0, 1, key.ctypes.data, idx.ctypes.data, stream) == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(3):
        ev[0].record()
        assert L.wg_gpu_seal_strided(h, n, P, 0, 0, pt.data_ptr() + 16, S, wire.data_ptr(), S, st.data_ptr(), stream) == 0
        ev[1].record()
        assert L.wg_gpu_open_strided(h, n, P + 32, 0, wire.data_ptr(), S, back.data_ptr() + 16, S, st.data_ptr(), stream) == 0
        ev[2].record()
        torch.cuda.synchronize()
        print(f"seal {ev[0].elapsed_time(ev[1]):.3f} ms  open {ev[1].elapsed_time(ev[2]):.3f} ms")
    buf = np.zeros((2, BLOCKS, ROUNDS, PHASES), np.uint64)
    assert L.wg_gpu_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
    for seal, name in ((1, "seal"), (0, "open")):
        s = buf[seal].astype(np.int64)
        used = (s[:, 0, 0] != 0)
        s = s[used]
        nr = int((s[0, :, 0] != 0).sum())
        print(f"{name}: {used.sum()} workgroups stamped, {nr} rounds")
        print("round " + " ".join(f"{x:>13s}" for x in NAMES))
        for r in range(nr):
            d = []
            for ph in range(PHASES):
                if ph < PHASES - 1:
                    v = s[:, r, ph + 1] - s[:, r, ph]
                elif r + 1 < nr:
                    v = s[:, r + 1, 0] - s[:, r, ph]
                else:
                    v = np.zeros(1)
                d.append(np.median(v))
            print(f"{r:5d} " + " ".join(f"{x:13.0f}" for x in d))
        tot = s[:, nr - 1, 5] - s[:, 0, 0]
        print(f"  whole loop: median {np.median(tot):.0f} cycles per workgroup; "
              f"span of all stamps {s[:, :nr].max() - s[:, 0, 0].min()} cycles")


if __name__ == "__main__":
    main()
