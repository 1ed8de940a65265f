"""CPU check of the restructured algorithm the kernels implement: the float64 model of
passes A-E and finalizes 1-5 in tests/restructured_model.py -- spatial-first FIR, BN1 statistics from
the lag-Gram of x and window sums, BN2/BN3 statistics and every weight gradient from per-trial
partial sums -- equals the float64 oracle (itself pinned to the reference's golden vectors) to
rounding, on the golden shapes (incl. T = 257, EEGNet-16,4, dropout) and on inputs with a DC offset."""

from __future__ import annotations

import numpy as np
import pytest

import restructured_model as rm
from golden_util import Golden, PARAM_NAMES
from oracle import numpy_ref as nr


def _compare(params, bufs, x, y, p=0.0, masks=None):
    logits, cache, _ = nr.forward(params, bufs, x, train=True, p=p, masks=masks)
    _, dl = nr.cross_entropy(logits, y)
    ref = nr.backward(cache, dl)
    out = rm.step(params, bufs, x, labels=y, p=p, masks=masks)
    np.testing.assert_allclose(out["logits"], logits, rtol=1e-10, atol=1e-12)
    scale = max(float(np.abs(v).max()) for v in ref.values())
    for k in PARAM_NAMES:
        np.testing.assert_allclose(out["grads"][k], ref[k], rtol=1e-8, atol=1e-10 * scale, err_msg=k)


@pytest.mark.parametrize("name", ["G1", "G2", "G4", "G5_F16D4", "G5_8x64", "G6"])
def test_restructured_equals_oracle_on_golden_shapes(name):
    g = Golden(name)
    _compare(g.init_params(), g.init_buffers(), g.x, g.y, g.meta["p"], g.masks(0))


def test_restructured_equals_oracle_with_dc_offset():
    g = Golden("G1")
    _compare(g.init_params(), g.init_buffers(), g.x + 5.0, g.y)
