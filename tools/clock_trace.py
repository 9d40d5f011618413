#!/usr/bin/env python3
"""Per-step in-kernel shader clock of the config-2 seal from a cold start
(diagnostic build: make -C neptun_amd/csrc variant NAME=stamp DEFS=-DWG_STAMP=1).

    python tools/clock_trace.py build/variants/libneptun_gpu_stamp.so OUT.json

Each step = seal + open of 1M x 1350 B (the bench's shapes).  After every seal the
stamp arrays are snapshotted on the device (no host sync between steps); the clock
of a step is the median over workgroups of d(s_memtime) / d(s_memrealtime) x 100 MHz
between rounds 0 and 10 of the last group each workgroup sealed.  Phases: A = the
first steps of the process (after input generation), B = after 1 s idle, C = after
1 s idle then ~50 ms of device copies (a different load).
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.ab import bind  # noqa: E402

BLOCKS, ROUNDS, PHASES = 4096, 16, 6


def main():
    import torch
    from tools import synth
    L = bind(sys.argv[1])
    L.wg_gpu_debug_snapshot.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
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
    words = 2 * BLOCKS * ROUNDS * PHASES + 2 * BLOCKS * ROUNDS
    steps_per_phase = {"A_cold": 40, "B_after_idle": 25, "C_after_other_load": 25}
    snaps = torch.zeros((sum(steps_per_phase.values()), words), dtype=torch.int64, device=dev)
    scratch = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
    out = {"what": __doc__.strip().splitlines()[0], "phases": {}}
    k = 0
    for phase, steps in steps_per_phase.items():
        if phase != "A_cold":
            torch.cuda.synchronize()
            time.sleep(1.0)
        if phase == "C_after_other_load":
            for _ in range(100):  # ~50 ms of 256 MiB device copies
                scratch.copy_(wire[: scratch.numel()])
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        for i in range(steps):
            evs[i][0].record()
            assert L.wg_gpu_seal_strided(h, n, P, 0, 0, pt.data_ptr() + 16, S, wire.data_ptr(), S,
                                         st.data_ptr(), stream) == 0
            evs[i][1].record()
            assert L.wg_gpu_debug_snapshot(snaps[k + i].data_ptr(), stream) == 0
            assert L.wg_gpu_open_strided(h, n, P + 32, 0, wire.data_ptr(), S, back.data_ptr() + 16, S,
                                         st.data_ptr(), stream) == 0
            evs[i][2].record()
        torch.cuda.synchronize()
        sn = snaps[k:k + steps].cpu().numpy().astype(np.int64)
        a = 2 * BLOCKS * ROUNDS * PHASES
        stamps = sn[:, :a].reshape(steps, 2, BLOCKS, ROUNDS, PHASES)[:, 1]   # seal
        rt = sn[:, a:].reshape(steps, 2, BLOCKS, ROUNDS)[:, 1]
        clocks = []
        for i in range(steps):
            t0, t1 = stamps[i, :, 0, 0], stamps[i, :, 10, 0]
            r0, r1 = rt[i, :, 0], rt[i, :, 10]
            ok = (t0 > 0) & (t1 > t0) & (r1 > r0)
            clocks.append(float(np.median((t1[ok] - t0[ok]) / (r1[ok] - r0[ok]) * 100.0)) if ok.any() else None)
        out["phases"][phase] = {
            "seal_ms": [round(e[0].elapsed_time(e[1]), 4) for e in evs],
            "open_ms": [round(e[1].elapsed_time(e[2]), 4) for e in evs],
            "seal_clock_MHz": [round(c, 1) if c else None for c in clocks],
        }
        print(phase, json.dumps(out["phases"][phase]), flush=True)
        k += steps
    ok = int(st.abs().sum()) == 0 and torch.equal(back.view(n, S)[:, 16:16 + P], pt.view(n, S)[:, 16:16 + P])
    out["round_trip_ok"] = ok
    with open(sys.argv[2], "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
