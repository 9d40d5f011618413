"""CPU stand-in for bench.py's GPU workload -- test support only (not a test module).

Same interface as bench.StridedWorkload; rank r sleeps (r+1) ms per step.  Used in
process by tests/test_bench_dist.py and, through bench.py's BENCH_FAKE_DEVICE hook,
by the `bench.py --gpus N` self-launch tests (the ranks are real child processes).
"""
import os
import time


class CpuEvent:
    def __init__(self):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def cpu_device(local):
    return "cpu", None, (lambda: None), CpuEvent


class FakeWorkload:
    def __init__(self, args, dev, rank, world):
        self.rank = rank
        self.packets = 1000 * (rank + 1)
        self.payload_bytes = 1350 * self.packets
        self.launch_bytes = {"seal": 2732 * self.packets, "open": 2732 * self.packets}
        self.kernels = {"seal": "fake_seal", "open": "fake_open"}
        self.fail = os.environ.get("FAKE_FAIL_RANK") == str(rank)
        self.crash = os.environ.get("FAKE_CRASH_RANK") == str(rank)

    def step(self, stream, evs=None):
        if self.crash:
            os._exit(7)  # a rank that dies before the barrier
        if evs:
            evs[0].record()
        time.sleep(0.001 * (self.rank + 1))
        if evs:
            evs[1].record()
        time.sleep(0.0005)
        if evs:
            evs[2].record()

    def verify(self):
        return not self.fail

    def describe(self, world):
        return {"workload": "fake", "parallelism": f"{world} shard(s), no collective"}

    def close(self):
        pass
