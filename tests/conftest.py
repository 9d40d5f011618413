import gc
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the HIP runtime's error log (level 1: errors only) on stderr, which pytest shows with
# a failing test: a GPU memory fault then names its address and the faulting agent
os.environ.setdefault("AMD_LOG_LEVEL", "1")
# Device-to-host copies into pageable memory (every tensor.cpu() here) take the HIP
# runtime's staged path at every size.  From 1 MiB the runtime otherwise locks the
# pageable destination on the fly ("Locking to pool", tools/probes/d2h_path.py) and the
# copy engine writes the user pages directly; both hipErrorIllegalAddress failures of
# the suite (GPUTEST_r05: a 1,664,064-byte back.cpu(); r06h: a 4,386,816-byte
# d_dst.cpu()) were raised inside such a copy, after a clean device synchronize
# (DESIGN.md §6).  The library's own copies land in pinned staging or registered
# memory (the host pipe asks its callers for pinned buffers, neptun_gpu.h).
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "1000000")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def pytest_unconfigure(config):
    # a process that does not exit within a minute of the session's end dumps every
    # thread's Python stack and exits (a hang at interpreter or runtime teardown)
    import faulthandler
    faulthandler.dump_traceback_later(60, exit=True)


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


@pytest.fixture(autouse=True)
def _gpu_fault_attribution(request):
    """A GPU memory fault is reported asynchronously, at some later HIP call.  After
    every gpu test: collect the test's garbage (Tunns, engines and contexts left in
    reference cycles are destroyed here, not by a collection during a later test),
    drain the device and make one device-to-host copy, so a fault surfaces in the
    teardown of the test whose work caused it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return
    gc.collect()
    torch.cuda.synchronize()
    torch.ones(1, device="cuda").cpu()
