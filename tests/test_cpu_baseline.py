"""CPU baseline harness (bench.py's cpu_baseline leg, oracle/cpu_baseline.c): pinned
per-thread workers, the scaling curve and the labels of the all-core figure."""
import json
import os
import subprocess

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "build", "cpu_baseline")


def _run(*args):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return subprocess.run([EXE, *args], capture_output=True, text=True, timeout=120)


def test_pinned_per_thread_round_trip_is_clean():
    out = _run("--impl", "openssl", "--threads", "2", "--packets-per-thread", "2048", "--reps", "3", "--pin")
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert d["pinned"] is True and d["packets"] == 4096 and d["tag_failures"] == 0 and d["gbps"] > 0


def test_oracle_impl_round_trip_is_clean():
    out = _run("--impl", "oracle", "--threads", "1", "--packets", "512", "--reps", "1")
    assert out.returncode == 0, out.stderr
    assert json.loads(out.stdout)["tag_failures"] == 0


def test_pin_refuses_more_threads_than_physical_cores():
    n = len(os.sched_getaffinity(0))
    out = _run("--threads", str(4 * n + 1), "--packets-per-thread", "16", "--reps", "1", "--pin")
    assert out.returncode == 2 and "physical cores" in out.stderr


def test_cpu_baseline_fields():
    cpus = bench.host_cpus()
    t = max(1, min(2, cpus["physical_cores"], cpus["allowed_cpus"]))
    d = bench.cpu_baseline(t, cpus, [1])
    assert d["threads_at_share"] == t and d["kind"] == "port" and d["value"] > 0
    assert set(d["threads_gbps"]) == {"1", str(t)} and d["scaling_efficiency"]["1"] == 1.0
    # value: the best measured thread count, its point beside the share's
    assert d["value"] == max(d["threads_gbps"].values()) and d["threads_gbps"][str(d["cores"])] == d["value"]
    assert d["value_at_share"] == d["threads_gbps"][str(t)]
    if t >= cpus["physical_cores"]:
        assert d["all_physical_cores_gbps"] == d["value_at_share"]
    else:
        assert d["all_physical_cores_extrapolated_gbps"] > 0
        assert d["all_physical_cores_upper_bound_gbps"] >= d["all_physical_cores_extrapolated_gbps"] * 0.999


def test_cpu_baseline_at_the_reference_bench_sizes():
    """--size P --op seal: the CPU baseline runs P-byte packets and reports the seal rate
    (the reference's chacha20poly1305_benching.rs shape), with the same payload bytes per
    worker as config 1."""
    cpus = bench.host_cpus()
    d = bench.cpu_baseline(1, cpus, [], size=8192, op="seal")
    assert d["size"] == 8192 and d["op"] == "seal" and d["value"] == d["seal_gbps"] > 0
    assert "8192 B" in d["sample"] and "best seal time" in d["sample"]
