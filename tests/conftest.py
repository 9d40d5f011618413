import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this container")
    return torch


@pytest.fixture(scope="session")
def gpu(torch_cuda):
    """Session-wide context with a 4096-slot key table (config 4 size)."""
    from neptun_amd import GpuContext  # raises loudly if the .so is missing
    ctx = GpuContext(0, key_slots=4096)
    yield ctx
    ctx.close()
