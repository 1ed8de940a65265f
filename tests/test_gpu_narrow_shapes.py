"""GPU parity of the F2 <= 16 step at shapes the golden fixtures do not reach: F2 = 4, 8, 12 (the row
guards of the runtime-shape passes, e.g. k_pass_dr's rows o >= F2 and its zero row buffers), T/4 not a
multiple of 64 and T/32 * 8 < T/4 (pool truncation inside a lane chunk), T/4 = 200 (four lane chunks
per row: the lane-shift carries of the transposed conv and of dw2), D = 1, and odd batches (a ghost
trial at the end of a workgroup's trial pair in k_pass_dr).

Per shape: the module path (forward_train + backward kernels) with injected masks against the float64
oracle step (reference model.py:91-99 forward, model.py:147 backward, clamps model.py:44 / 84), and the
fused step (on-device masks, CE, backward, clamps, Adam) against the oracle given the restated device
masks.  Tolerance: north_star's rtol 1e-4, atol 1e-5 * max|ref| (tests/golden_util.py)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from golden_util import assert_close, assert_grads_close, assert_params_close, make_inputs, make_masks
from hip_cases import device_masks, random_model
from test_gpu_wide import _step

pytestmark = pytest.mark.gpu

SHAPES = [
    # C, T, F1, D, B, p
    (22, 256, 4, 2, 13, 0.5),       # F2 = 8 at the benchmark's C x T (runtime instantiation), odd batch
    (16, 200, 2, 2, 9, 0.25),       # F2 = 4, T1 = 50, T2 = 6 (48 pooled samples of 50)
    (22, 257, 6, 2, 11, 0.5),       # F2 = 12 at the recordings' T (runtime instantiation)
    (8, 100, 4, 1, 7, 0.5),         # F2 = 4, D = 1, T1 = 25
    (4, 800, 8, 2, 5, 0.25),        # F2 = 16, T1 = 200: four 64-lane chunks per row (the last partial)
]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.mark.parametrize("C,T,F1,D,B,p", SHAPES)
def test_narrow_shape_module_step_matches_oracle(C, T, F1, D, B, p):
    m = random_model(C, T, F1=F1, D=D, p=p, seed=7 * C + T + F1)
    x_np, y_np = make_inputs(B, C, T, 900 + T)
    masks = make_masks(B, F1 * D, T, 910 + C, p)
    _step(m, x_np, y_np, p, masks, f"EEGNet-{F1},{D} {C}x{T} B={B}")


@pytest.mark.parametrize("C,T,F1,D,B,p", SHAPES)
def test_narrow_shape_fused_step_matches_oracle(C, T, F1, D, B, p):
    from eegnetreplication_amd import FusedTrainer
    from oracle import numpy_ref as nr
    dev = _dev()
    m = random_model(C, T, F1=F1, D=D, p=p, seed=11 * C + T + D)
    x_np, y_np = make_inputs(B, C, T, 700 + T)
    params = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.named_parameters()}
    bufs = {k: v.detach().cpu().numpy() for k, v in m.named_buffers()}
    seed, offset = 0x51DE_5EED, 5
    masks = device_masks(B, F1 * D, T, seed, offset, p)
    ref = nr.train_step(params, bufs, x_np, y_np, nr.adam_init(params), p=p, masks=masks)
    model = m.to(dev).train()
    model.next_dropout_key = lambda: (seed, offset)
    tr = FusedTrainer(model, lr=1e-3, eps=1e-7)
    x = torch.from_numpy(np.ascontiguousarray(x_np, dtype=np.float32)).to(dev)
    y = torch.from_numpy(y_np).to(dev)
    logits = torch.empty((B, 4), device=dev)
    loss = tr.step(x, y, logits=logits)
    what = f"fused EEGNet-{F1},{D} {C}x{T} B={B}"
    assert_close(logits.cpu().numpy(), ref["logits"], name=f"{what} logits")
    assert abs(float(loss) - float(ref["loss"])) <= 1e-4 * max(1.0, abs(float(ref["loss"]))), what
    n = 0
    gr = {}
    for k, prm in model.named_parameters():
        gr[k] = tr.adam.grads[n:n + prm.numel()].view(prm.shape).cpu().numpy()
        n += prm.numel()
    assert_grads_close(gr, ref["grads"], prefix=f"{what} grad.")
    assert_params_close({k: prm.detach().cpu().numpy() for k, prm in model.named_parameters()},
                        ref["params"], prefix=f"{what} step1.")
