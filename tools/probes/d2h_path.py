"""Which path the HIP runtime takes for a device-to-host copy into pageable memory
(AMD_LOG_LEVEL=4 prints "HSA Copy Using Pinned / Staging resource"), and its rate.
Pageable destinations of >= 1 MiB are locked on the fly ("Locking to pool") and
written by the copy engine; GPU_PINNED_MIN_XFER_SIZE (MiB) raises that threshold.
(the test harness's copies.)"""
import time

import torch

for n in (300_000, 1_660_000, 4_386_816, 40_000_000, 400_000_000):
    x = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    print("=== D2H", n, flush=True)
    t0 = time.perf_counter()
    y = x.cpu()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"=== done {n} {dt * 1e3:.2f} ms {n / dt / 1e9:.2f} GB/s", flush=True)
    del x, y
