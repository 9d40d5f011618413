"""The compute (VALU-issue) roofline the bench line carries (tools/compute_roofline.py,
bench.compute_roofline): the instruction model stays at or below what the committed
PMC runs counted, and the floor is priced at the line's own live clock."""
import json
import os

import pytest

import bench
from tools import compute_roofline as cr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc_per_64(config, kernel, packets):
    d = json.load(open(os.path.join(ROOT, "profiles", f"pmc_valu_config{config}.json")))
    k = d["kernels"][kernel]
    return k["valu_per_wave"] * k["waves"] * 64 / packets


@pytest.mark.parametrize("kernel", ["aead_strided_kernel<true, false>", "aead_strided_kernel<false, false>"])
def test_model_is_a_floor_of_the_measured_instructions_config2(kernel):
    model = cr.launch_floor((1350, 1 << 20))["model_valu_instr_per_64_packets"]
    measured = pmc_per_64(2, kernel, 1 << 20)
    assert model <= measured <= 1.03 * model, (model, measured)


@pytest.mark.parametrize("seal", [True, False])
def test_model_is_a_floor_config4_per_lane_keys(seal):
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_valu_config4.json")))["kernels"]
    kernel = [k for k in d if k.endswith("<true>" if seal else "<false>")][0]
    model = cr.launch_floor((1350, 1 << 24), per_lane_keys=True)["model_valu_instr_per_64_packets"]
    assert model <= pmc_per_64(4, kernel, 1 << 24)


def test_floor_scales_with_the_clock():
    a = cr.launch_floor((1350, 1 << 20), 2.4)
    b = cr.launch_floor((1350, 1 << 20), 1.944)
    assert a["floor_ms_at_clock"] == pytest.approx(a["floor_ms_at_2p4GHz"], abs=1e-4)
    assert b["floor_ms_at_clock"] == pytest.approx(a["floor_ms_at_2p4GHz"] * 2.4 / 1.944, rel=1e-3)


def test_bench_prices_the_floor_at_the_live_clock():
    class Wl:
        packets = 1 << 20
        profile_tag = "config2"

        def size_hist(self):
            return {1350: self.packets}

    out = bench.compute_roofline(Wl(), "aead_strided_kernel<false, false>", 0.7214, 1.9638, 0.69)
    floor = cr.launch_floor({1350: 1 << 20}, 1.9638)["floor_ms_at_clock"]
    assert out["clock_GHz_live"] == pytest.approx(1.9638)
    assert out["frac"] == pytest.approx(floor / 0.7214, abs=1e-4)
    assert out["frac_sustained"] == pytest.approx(floor / 0.69, abs=1e-4)
    # the PMC run's own clock only as frac_in_profiled_run
    assert "frac_in_profiled_run" in out and out["clock_GHz_profiled"] != out["clock_GHz_live"]
    # no live clock (no amd-smi): no frac at all rather than one at a stale clock
    assert "frac" not in bench.compute_roofline(Wl(), "aead_strided_kernel<false, false>", 0.72, None)
