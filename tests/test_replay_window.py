"""The C++ replay window (wg_replay_*, neptun_amd/csrc/wg_tunn.cpp) against the
reference's own test and against the Python restatement of session.rs:40-157.
Runs on CPU: the window is host code."""
import random

import pytest

from neptun_amd.tunn import ReplayWindow
from oracle.tunn_model import N_BITS, Replay

INVALID_COUNTER, DUPLICATE_COUNTER = 11, 12


@pytest.mark.parametrize("impl", ["cpp", "model"])
def test_reference_replay_counter_test(impl):
    """session.rs:367-414 (test_replay_counter), statement by statement."""
    c = ReplayWindow() if impl == "cpp" else Replay()
    ok = lambda r: r == 0  # noqa: E731
    assert ok(c.mark_did_receive(0)) and not ok(c.mark_did_receive(0))
    assert ok(c.mark_did_receive(1)) and not ok(c.mark_did_receive(1))
    assert ok(c.mark_did_receive(63)) and not ok(c.mark_did_receive(63))
    assert ok(c.mark_did_receive(15)) and not ok(c.mark_did_receive(15))
    for i in range(64, N_BITS + 128):
        assert ok(c.mark_did_receive(i)) and not ok(c.mark_did_receive(i))
    assert ok(c.mark_did_receive(N_BITS * 3))
    for i in range(0, N_BITS * 2 + 1):
        assert c.will_accept(i) == INVALID_COUNTER
        assert not ok(c.mark_did_receive(i))
    for i in range(N_BITS * 2 + 1, N_BITS * 3):
        assert ok(c.will_accept(i))
    assert c.will_accept(N_BITS * 3) == DUPLICATE_COUNTER
    for i in reversed(range(N_BITS * 2 + 1, N_BITS * 3)):
        assert ok(c.mark_did_receive(i)) and not ok(c.mark_did_receive(i))
    for d in (70, 71, 72, 72 + 125, 63):
        assert ok(c.mark_did_receive(N_BITS * 3 + d))
    for d in (70, 71, 72):
        assert not ok(c.mark_did_receive(N_BITS * 3 + d))


@pytest.mark.parametrize("seed", range(6))
def test_cpp_window_equals_model_on_random_traffic(seed):
    rng = random.Random(seed)
    a, b = ReplayWindow(), Replay()
    ctr = 0
    for _ in range(20000):
        r = rng.random()
        if r < 0.6:
            ctr += 1
            x = ctr
        elif r < 0.8:
            x = max(0, ctr - rng.randrange(0, 1200))  # reorder / replay inside and past the window
        elif r < 0.95:
            ctr += rng.randrange(1, 3000)  # loss bursts, incl. jumps past N_BITS
            x = ctr
        else:
            x = rng.getrandbits(64) if rng.random() < 0.1 else ctr + rng.randrange(0, 70)
        assert a.will_accept(x) == b.will_accept(x)
        assert a.mark_did_receive(x) == b.mark_did_receive(x)
        assert a.w.next == b.next
        assert list(a.w.bitmap) == b.bitmap
