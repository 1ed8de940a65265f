"""cfg4 (BASELINE configs[3]: data-parallel synthetic batch 65536) at its own size on one GPU.

* The HIP step at B = 65536 against the float64 reference layer stack (oracle/torch_ref.py, stock
  ATen on the device) through a size-independent property: the batch is the cfg2 batch (4,096
  trials) tiled 16 times, masks included.  Batch statistics, the batch-mean loss and every gradient
  of the tiled batch equal those of one tile in exact arithmetic, so the B = 65536 result is held at
  north_star's rtol 1e-4 to the float64 reference run on one tile (a float64 stock-ATen run of all
  65,536 trials does not fit the test's time budget).  The only size-dependent term, the unbiased
  running variance n / (n - 1), is corrected for exactly.
* ``DataParallelTrainer`` (the cfg4 product path: local step, one all-reduce, clamp, Adam) at
  world 1 and B = 65536 is bit-identical to ``FusedTrainer`` over 3 steps on random data with the
  device dropout generator (same keys).

Reference semantics: the step model.py:141-148, the clamps model.py:44,84 after the reduction
(SURVEY F2), Adam train.py:94-101.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from golden_util import PARAM_NAMES, assert_close, assert_grads_close, make_inputs, make_masks
from hip_cases import grads_of, random_model

pytestmark = pytest.mark.gpu

B4, TILES, C, T = 4096, 16, 22, 256


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def test_cfg4_batch_65536_matches_float64_reference_by_tiling():
    from oracle import torch_ref as tr
    dev = _dev()
    B = B4 * TILES
    m = random_model(C, T, p=0.5, seed=3, perturb_bn=True).to(dev).train()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    x_np, y_np = make_inputs(B4, C, T, 4321)
    m2, m3 = make_masks(B4, 16, T, 77, 0.5)
    x1, y1 = torch.from_numpy(x_np).to(dev), torch.from_numpy(y_np).to(dev)
    mk1 = (torch.from_numpy(m2).to(dev), torch.from_numpy(m3).to(dev))
    x, y = x1.repeat(TILES, 1, 1), y1.repeat(TILES)
    m.set_dropout_masks(mk1[0].repeat(TILES, 1, 1), mk1[1].repeat(TILES, 1, 1))
    logits = m(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    torch.cuda.synchronize()
    got_logits = logits.detach().view(TILES, B4, 4)
    # every tile sees the same batch statistics: identical logits, bit for bit
    assert torch.equal(got_logits, got_logits[:1].expand_as(got_logits))

    ref = tr.TorchRefEEGNet(state, p=0.5, device=dev, dtype=torch.float64)
    rl = ref(x1.double(), mk1)
    rloss = torch.nn.functional.cross_entropy(rl, y1)
    rloss.backward()
    assert_close(got_logits[0].cpu().numpy(), rl.detach().cpu().numpy(), name="B65536 logits")
    assert abs(float(loss) - float(rloss)) <= 1e-4 * max(1.0, abs(float(rloss)))
    assert_grads_close(grads_of(m), {k: ref.params[k].grad.cpu().numpy() for k in PARAM_NAMES},
                       prefix="B65536 grad.")
    # running statistics: the mean is size-independent; the variance's unbiasing factor n / (n - 1)
    # is for n = B * (elements per trial and channel)
    per = {"temporal.1": C * T, "aggregation.0": T, "block_2.2": T // 4}
    for k, b in m.named_buffers():
        got = b.detach().cpu().numpy()
        r = ref.buffers[k].cpu().numpy()
        pre = k.rsplit(".", 1)[0]
        if k.endswith("running_mean"):
            assert_close(got, r, atol_abs=1e-5 * max(1.0, float(np.abs(r).max())), name=k)
        elif k.endswith("running_var"):
            n1, nB = float(B4 * per[pre]), float(B * per[pre])
            rv0 = state[k].astype(np.float64)
            biased = (r - 0.9 * rv0) / 0.1 * (n1 - 1.0) / n1
            assert_close(got, 0.9 * rv0 + 0.1 * biased * nB / (nB - 1.0), name=k)
        else:
            assert int(got) == int(state[k]) + 1, k


def test_cfg4_dp_world1_bit_identical_to_fused_at_65536():
    from eegnetreplication_amd import FusedTrainer
    from eegnetreplication_amd.distributed import DataParallelTrainer
    dev = _dev()
    B = B4 * TILES
    a = random_model(C, T, p=0.5, seed=5).to(dev).train()
    b = random_model(C, T, p=0.5, seed=5).to(dev).train()
    g = torch.Generator(device=dev).manual_seed(11)
    dp, fu = DataParallelTrainer(a), FusedTrainer(b)
    keys = iter([(0x5EED_0000 + s, s) for s in range(1, 10)])     # the DP trainer's keys at world 1
    b.next_dropout_key = lambda: next(keys)
    for s in range(3):
        x = torch.randn(B, C, T, device=dev, generator=g)
        y = torch.randint(0, 4, (B,), device=dev, generator=g)
        la = float(dp.step(x, y))
        lb = float(fu.step(x, y))
        assert la == lb and np.isfinite(la), s
    torch.cuda.synchronize()
    assert torch.equal(a.flat_parameters(), b.flat_parameters())
    assert torch.equal(a.flat_bn_buffers(), b.flat_bn_buffers())
    assert torch.equal(dp.adam.state, fu.adam.state)
    assert torch.equal(a.flat_num_batches_tracked(), b.flat_num_batches_tracked())
    assert int(dp.adam.step.item()) == 3
