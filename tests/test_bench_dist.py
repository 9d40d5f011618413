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
from bench_fake import FakeWorkload, cpu_device


def _worker(rank, world, port, outdir, fail_rank, device_count=None):
    import contextlib
    import io
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fail_rank is not None:
        os.environ["FAKE_FAIL_RANK"] = str(fail_rank)
    import bench
    args = bench.parse(["--gpus", str(world), "--steps", "5", "--warmup", "1", "--no-cpu-baseline", "--sustain-seconds", "0.05"])
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


def _bench_cli(args, extra_env=None, timeout=120):
    """Run `python bench.py ...` as a real command (the driver's form) with the CPU
    stand-in injected through BENCH_FAKE_DEVICE; returns (rc, stdout lines)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BENCH_FAKE_DEVICE"] = "tests.bench_fake"
    env.update(extra_env or {})
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], cwd=root, env=env,
                         capture_output=True, text=True, timeout=timeout)
    return out.returncode, [x for x in out.stdout.splitlines() if x.startswith("{")]


COMMON = ["--steps", "5", "--warmup", "1", "--no-cpu-baseline", "--sustain-seconds", "0.05"]


def test_gpus_flag_starts_that_many_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes
    itself and prints ONE line for both: n_gpus 2, two per_rank entries, the slower
    rank's time, the two shards' payload summed."""
    rc, lines = _bench_cli(["--gpus", "2", *COMMON])
    assert rc == 0 and len(lines) == 1, lines
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and len(line["per_rank"]) == 2
    assert [r["rank"] for r in line["per_rank"]] == [0, 1]
    assert line["packets_per_step"] == 3000 and line["ms_per_step"] >= 2.5


def test_gpus_flag_one_is_a_single_rank():
    rc, lines = _bench_cli(["--gpus", "1", *COMMON])
    assert rc == 0 and len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and "per_rank" not in line


def test_gpus_flag_and_launcher_world_must_agree():
    """A launcher's WORLD_SIZE that differs from --gpus is refused with an error line."""
    rc, lines = _bench_cli(["--gpus", "8", *COMMON],
                           extra_env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2
    line = json.loads(lines[0])
    assert "error" in line and line["n_gpus"] == 1 and line["gpus_flag"] == 8


def test_gpus_flag_refuses_more_ranks_than_gpus():
    """--gpus 2 on a node with one visible GPU: the ranks refuse (rc 2, one error line)."""
    rc, lines = _bench_cli(["--gpus", "2", *COMMON], extra_env={"BENCH_FAKE_GPUS": "1"})
    assert rc == 2 and len(lines) == 1
    assert json.loads(lines[0])["visible_gpus"] == 1


def test_gpus_flag_a_dead_rank_ends_the_run():
    """A rank that dies before the start barrier does not leave the others waiting:
    the launcher stops them and exits non-zero."""
    t0 = time.time()
    rc, lines = _bench_cli(["--gpus", "2", *COMMON], extra_env={"FAKE_CRASH_RANK": "1"})
    assert rc != 0
    assert time.time() - t0 < 100


@pytest.mark.gpu
def test_gpus_flag_two_ranks_on_the_gpu(torch_cuda):
    """The N-rank path with the real workload and HIP kernels: `bench.py --gpus 2` starts
    two rank processes that both run on cuda:0 here (tests/bench_shared_gpu.py: a 1-GPU
    box has one device), each sealing and opening its own shard with disjoint counters,
    gloo carrying the barrier, max-over-ranks time and byte sums.  One line: n_gpus 2,
    both ranks' telemetry, both shards verified, the packets summed."""
    rc, lines = _bench_cli(["--gpus", "2", "--packets", "65536", *COMMON], timeout=300,
                           extra_env={"BENCH_FAKE_DEVICE": "tests.bench_shared_gpu", "BENCH_FAKE_GPUS": "2"})
    assert rc == 0 and len(lines) == 1, lines
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and len(line["per_rank"]) == 2
    assert line["packets_per_step"] == 2 * 65536
    assert "error" not in line and line.get("verified")
