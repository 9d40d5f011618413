"""GPU test support (not a test module): bench.py's multi-rank path with every rank on
cuda:0 -- the real workload and HIP kernels, gloo for the start barrier / max-over-ranks
time / byte sums -- so a 1-GPU box exercises the N-rank code end to end.  Loaded through
bench.py's BENCH_FAKE_DEVICE hook (which takes `FakeWorkload` and `cpu_device` names) by
tests/test_bench_dist.py; what it prints is test output, never a scaling number (the
ranks share one device)."""
import torch

import bench


def cpu_device(local):  # (the hook's name): every rank on device 0
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    return (dev, torch.cuda.current_stream(dev), lambda: torch.cuda.synchronize(dev),
            lambda: torch.cuda.Event(enable_timing=True))


FakeWorkload = bench.make_workload
