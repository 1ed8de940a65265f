"""bench.py's host-side arithmetic (no GPU): the implemented-FLOP / byte tables behind the roofline
lines, the roofline pricing, and the untimed-step rule ahead of the headline's timed region."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_cfg2_tables_match_the_reported_per_trial_totals():
    alg = bench.kernel_algorithmic(22, 256)
    assert set(alg) == {"k_pass_a", "k_pass_b", "k_pass_c", "k_pass_d", "k_pass_e"}
    assert sum(f for f, _ in alg.values()) == 1_749_632          # implemented_flop_per_trial
    assert sum(b for _, b in alg.values()) == 180_256            # implemented_bytes_per_trial
    ab = bench.kernel_alg_bytes(22, 256)
    assert ab["k_pass_a"] == ab["k_pass_e"] == 22 * 256 * 4      # x read by passes A and E
    assert sum(ab.values()) - ab["k_pass_c"] == bench.ALG_BYTES_PER_TRIAL


def test_cfg5_tables():
    alg = bench.kernel_algorithmic_wide(64, 512, 16, 4)
    assert sum(f for f, _ in alg.values()) == 20_852_736          # 20.9 MFLOP per trial


@pytest.mark.parametrize("fl,by,us", [(2.886e9, 92.3e6, 70.0), (1e6, 5e9, 100.0)])
def test_roofline_entry_takes_the_binding_roof(fl, by, us):
    e = bench.roofline_entry("k_pass_e", fl, by, 2 * by, us * 1e-6)
    t_f, t_b = fl / (bench.PEAK_FP32_TFLOPS * 1e12), by / (bench.PEAK_HBM_GBS * 1e9)
    assert e["bound"] == ("mfma" if t_f >= t_b else "hbm")
    assert e["frac"] == pytest.approx(max(t_f, t_b) / (us * 1e-6), rel=1e-3)
    assert e["fp32_frac"] == pytest.approx(t_f / (us * 1e-6), abs=1e-4)


@pytest.mark.parametrize("warmup,survey,prof,expect", [(5, 5, True, 49), (10, 5, True, 44), (3, 5, False, 57),
                                                        (60, 5, True, 0), (200, 5, True, 0)])
def test_untimed_steps_rule(warmup, survey, prof, expect):
    settle = bench.settle_steps(warmup, survey, prof)
    assert settle == expect
    assert warmup + (survey + 1 if prof else 0) + settle >= bench.MIN_UNTIMED
