"""The C ABI from plain C (examples/tunn_roundtrip.c): compiles against
include/*.h and links libneptun_gpu.so with gcc -- the shape of the Rust
binding in INTEGRATION.md.  CPU: builds and fails loudly without a device;
GPU: a full encapsulate -> decapsulate -> replay-rejection round trip."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(tmp_path):
    exe = str(tmp_path / "tunn_roundtrip")
    lib = os.path.join(ROOT, "neptun_amd")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "tunn_roundtrip.c"), "-L", lib, "-lneptun_gpu",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    return exe


def test_c_example_builds_and_fails_loudly_without_gpu(tmp_path):
    exe = build(tmp_path)
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu-marked test")
    r = subprocess.run([exe, "8"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_c_example_round_trip_on_gpu(tmp_path, torch_cuda):
    exe = build(tmp_path)
    r = subprocess.run([exe, "4096"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok: 4096 packets")
