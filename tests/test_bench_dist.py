"""bench.py's multi-rank path (one process per GPU, gloo control plane) on CPU.

The data path has no collective (packets shard independently);
what must hold across ranks is the timing contract: barrier + sync around the
timed steps, MAX of the elapsed time over ranks, SUM of the payload, and a
failed verification on any rank failing the run.  The GPU workload is replaced
by a CPU stand-in with the same interface; everything else is bench.run.
"""
import json
import os
import socket
import time

import pytest
import torch.multiprocessing as mp


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
    """Same interface as bench.StridedWorkload; rank r sleeps (r+1) ms per step."""

    def __init__(self, args, dev, rank, world):
        self.rank = rank
        self.packets = 1000 * (rank + 1)
        self.payload_bytes = 1350 * self.packets
        self.launch_bytes = {"seal": 2732 * self.packets, "open": 2732 * self.packets}
        self.kernels = {"seal": "fake_seal", "open": "fake_open"}
        self.fail = os.environ.get("FAKE_FAIL_RANK") == str(rank)

    def step(self, stream, evs=None):
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


def _worker(rank, world, port, outdir, fail_rank, device_count=None):
    import contextlib
    import io
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fail_rank is not None:
        os.environ["FAKE_FAIL_RANK"] = str(fail_rank)
    import bench
    args = bench.parse(["--steps", "5", "--warmup", "1", "--no-cpu-baseline", "--sustain-seconds", "0.05"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.run(args, factory=FakeWorkload, device_fn=cpu_device,
                       device_count=world if device_count is None else device_count)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"rc": rc, "out": buf.getvalue()}, f)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(tmp_path, world, fail_rank=None, device_count=None):
    mp.start_processes(_worker, args=(world, free_port(), str(tmp_path), fail_rank, device_count),
                       nprocs=world, join=True, start_method="spawn")
    return [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]


@pytest.mark.parametrize("world", [2])
def test_two_ranks_aggregate_max_time_and_sum_payload(tmp_path, world):
    res = run_ranks(tmp_path, world)
    assert all(r["rc"] == 0 for r in res)
    assert res[1]["out"] == ""  # only rank 0 prints
    line = json.loads(res[0]["out"])
    assert line["n_gpus"] == 2 and line["visible_gpus"] == 2 and line["scaling"] == "weak"
    assert line["packets_per_step"] == 1000 + 2000
    # the slowest rank (rank 1: >= 2.5 ms per step) sets the time
    assert line["ms_per_step"] >= 2.5
    total_payload = 1350 * 3000
    want = total_payload * 8 / (line["ms_per_step"] * 1e-3) / 1e9
    assert abs(line["value"] - want) / want < 1e-3
    assert line["config"]["parallelism"] == "2 shard(s), no collective"
    # every rank's own numbers travel with the line, so a sub-linear N-GPU result
    # can be attributed to a rank (its kernel times, its sustained rate and, on
    # GPUs, its own package's power / clock / PPT state)
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1] and [r["local_rank"] for r in pr] == [0, 1]
    assert pr[1]["kernel_ms"]["seal"] >= 1.9 and pr[0]["kernel_ms"]["seal"] < pr[1]["kernel_ms"]["seal"]
    assert [r["packets"] for r in pr] == [1000, 2000]
    assert max(r["elapsed_s"] for r in pr) * 1e3 / 5 == pytest.approx(line["ms_per_step"], rel=1e-3)
    assert all(r["sustained_gbps"] > 0 and r["sustained_kernel_ms"]["seal"] > 0 for r in pr)
    assert line["sustained"]["steps"] >= 1


def test_failed_verification_on_any_rank_fails_the_run(tmp_path):
    res = run_ranks(tmp_path, 2, fail_rank=1)
    assert all(r["rc"] == 1 for r in res)
    assert "error" in json.loads(res[0]["out"])


def test_more_ranks_than_gpus_is_refused(tmp_path):
    """An N-rank line must come from N distinct GPUs: 2 ranks on a 1-GPU node exit
    non-zero with an error line instead of publishing shared-device numbers."""
    res = run_ranks(tmp_path, 2, device_count=1)
    assert all(r["rc"] == 2 for r in res)
    line = json.loads(res[0]["out"])
    assert "error" in line and line["visible_gpus"] == 1 and line["n_gpus"] == 2
    assert res[1]["out"] == ""


def test_power_sampler_never_fails_the_bench(monkeypatch):
    """bench.PowerSampler reports what amd-smi gives and never raises: here (no GPU)
    the samples carry no busy GPU, or amd-smi errors out and the note says so."""
    import bench
    from tools import power_probe
    calls = []

    def fake_sample(gpu=0):
        calls.append(gpu)
        return {"err": "amd-smi: no GPU"} if len(calls) > 2 else {"gpu_data": []}

    monkeypatch.setattr(power_probe, "sample", fake_sample)
    s = bench.PowerSampler(period=0.01, gpu=3)
    s.start()
    time.sleep(0.2)
    out = s.stop()
    assert out.get("busy_samples") == 0 or "error" in out
    assert calls == [3, 3, 3]  # its own GPU; stops sampling at the first error


def test_smi_index_follows_visible_devices(monkeypatch):
    import bench
    for v in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.smi_index(5) == 5
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "6,7")
    assert bench.smi_index(1) == 7


def test_limiter_label_needs_the_power_limit():
    """roofline.limiter says 'package power' only when the mean socket power
    reaches the PPT limit (>= 1390 W), not whenever a sample flags PPT."""
    import bench
    pw = {"socket_power_W": 1397.0, "gfx_clock_MHz": 1963.8, "ppt_violation": ["ACTIVE"]}
    assert bench.power_limiter(pw).startswith("package power: 1397.0 W")
    assert bench.power_limiter(dict(pw, socket_power_W=1323.0)) is None
    assert bench.power_limiter(dict(pw, ppt_violation=["NOT ACTIVE"])) is None
    assert bench.power_limiter({}) is None
