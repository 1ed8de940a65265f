"""GPU parity of the F2 > 16 train step and fp32 eval (csrc/eegnet_wide.hip; BASELINE cfg5:
EEGNet-16,4 on 64ch x 512, reference model.py:13,21-84 with F1=16, D=4) beyond the two golden
fixtures (tests/test_gpu_parity.py G5_F16D4, G5_16x4_64x512):

* cfg5 train step against the float64 oracle with injected masks, and with the device generator;
* other wide shapes: F2 = 24 / 32 / 48 (a partial o-chunk, 2 and 3 chunks), T = 257, C = 22;
* the fused step (forward + CE + backward + clamps + Adam, 14,116 parameters through fin5's Adam
  loop) against the oracle step;
* cfg5 at B = 1024 against the reference layer stack in float64 on the device (size-independent
  check at a full batch);
* the fp32 wide eval kernel against the oracle.
Tolerance: north_star's rtol 1e-4, atol 1e-5 * max|ref| (tests/golden_util.py)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from golden_util import PARAM_NAMES, assert_close, assert_grads_close, assert_params_close, make_inputs, make_masks
from hip_cases import device_masks, flat_to_dict, grads_of, oracle_eval, oracle_step, random_model

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _step(m, x_np, y_np, p, masks, what):
    dev = _dev()
    ref_logits, ref_loss, ref_grads, ref_nb, _ = oracle_step(m, x_np, y_np, p=p, masks=masks)
    m = m.to(dev).train()
    if masks is not None:
        m.set_dropout_masks(torch.from_numpy(masks[0]).to(dev), torch.from_numpy(masks[1]).to(dev))
    x = torch.from_numpy(np.ascontiguousarray(x_np, dtype=np.float32)).to(dev)
    y = torch.from_numpy(y_np).to(dev)
    logits = m(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    assert_close(logits.detach().cpu().numpy(), ref_logits, name=f"{what} logits")
    assert abs(float(loss) - ref_loss) <= 1e-4 * max(1.0, abs(ref_loss)), f"{what} loss"
    assert_grads_close(grads_of(m), ref_grads, prefix=f"{what} grad.")
    bufs = {k: b.detach().cpu().numpy() for k, b in m.named_buffers()}
    for k, v in ref_nb.items():
        if "running_mean" in k:
            assert_close(bufs[k], v, atol_abs=1e-5 * max(1.0, float(np.abs(v).max())), name=f"{what} {k}")
        elif "running_var" in k:
            assert_close(bufs[k], v, name=f"{what} {k}")
        else:
            assert int(bufs[k]) == int(v), f"{what} {k}"
    return m


@pytest.mark.parametrize("C,T,F1,D,B,p", [
    (64, 512, 16, 4, 24, 0.25),     # cfg5
    (22, 257, 16, 4, 16, 0.5),      # F2 = 64 at the protocol shape (pool truncation)
    (22, 256, 12, 2, 16, 0.5),      # F2 = 24: one full + one partial o-chunk, F2P = 32
    (32, 256, 8, 4, 16, 0.25),      # F2 = 32
    (40, 128, 12, 4, 16, 0.5),      # F2 = 48: 3 chunks, F2P = 64, C = 40
])
def test_wide_train_step_matches_oracle(C, T, F1, D, B, p):
    m = random_model(C, T, F1=F1, D=D, p=p, seed=C + T + F1 * D)
    x_np, y_np = make_inputs(B, C, T, 500 + C)
    masks = make_masks(B, F1 * D, T, 500 + T, p)
    m = _step(m, x_np, y_np, p, masks, f"EEGNet-{F1},{D} {C}x{T}")
    m.eval()
    with torch.no_grad():
        out = m(torch.from_numpy(x_np).to(_dev())).cpu().numpy()
    assert_close(out, oracle_eval(m, x_np), name=f"EEGNet-{F1},{D} {C}x{T} eval")


def test_wide_dropout_generator_matches_restatement():
    """cfg5 with masks drawn on the device: the oracle given the restated masks agrees."""
    from eegnetreplication_amd import ops
    dev = _dev()
    B, C, T, p = 16, 64, 512, 0.25
    m = random_model(C, T, F1=16, D=4, p=p, seed=3)
    x_np, y_np = make_inputs(B, C, T, 8)
    seed, offset = 424242, 5
    masks = device_masks(B, 64, T, seed, offset, p)
    ref_logits, ref_loss, ref_grads, _, _ = oracle_step(m, x_np, y_np, p=p, masks=masks)
    m = m.to(dev).train()
    shape = m.shape
    flat, bn = m.flat_parameters().clone(), m.flat_bn_buffers().clone()
    ws = ops.new_workspace(shape, B, dev)
    x, y = torch.from_numpy(x_np).to(dev), torch.from_numpy(y_np).to(dev)
    logits = ops.forward_train(shape, flat, bn, x, ws, seed, offset)
    loss = torch.zeros(1, device=dev)
    grads = ops.backward(shape, flat, x, ws, seed, offset, labels=y, loss=loss)
    torch.cuda.synchronize()
    assert_close(logits.cpu().numpy(), ref_logits, name="cfg5 generator logits")
    assert abs(float(loss) - ref_loss) <= 1e-4 * max(1.0, abs(ref_loss))
    assert_grads_close(flat_to_dict(m, grads), ref_grads, prefix="cfg5 generator grad.")


def test_wide_fused_step_matches_oracle_adam():
    """eegnet_train_step at cfg5 (p = 0): logits, loss, grads and the post-Adam parameters (fin5's
    Adam covers all 14,116 parameters) against the oracle's train step."""
    from eegnetreplication_amd import FusedTrainer
    from oracle import numpy_ref as nr
    from hip_cases import state_np
    dev = _dev()
    B, C, T = 16, 64, 512
    m = random_model(C, T, F1=16, D=4, p=0.0, seed=12)
    params, bufs = state_np(m)
    x_np, y_np = make_inputs(B, C, T, 77)
    out = nr.train_step(params, bufs, x_np, y_np, nr.adam_init(params), p=0.0)
    m = m.to(dev).train()
    tr = FusedTrainer(m)
    logits = torch.empty(B, 4, device=dev)
    loss = tr.step(torch.from_numpy(x_np).to(dev), torch.from_numpy(y_np).to(dev), logits=logits)
    torch.cuda.synchronize()
    assert m.flat_parameters().numel() == 14116
    assert_close(logits.cpu().numpy(), out["logits"], name="cfg5 fused logits")
    assert abs(float(loss) - out["loss"]) <= 1e-4 * max(1.0, abs(out["loss"]))
    assert_grads_close(flat_to_dict(m, tr.adam.grads), out["grads"], prefix="cfg5 fused grad.")
    assert_params_close({k: p.detach().cpu().numpy() for k, p in m.named_parameters()}, out["params"],
                        prefix="cfg5 fused step1.")


def test_cfg5_full_batch_against_float64():
    """cfg5 at B = 1024 (p = 0.25, injected masks): logits, loss, all 12 grads and the running
    statistics against the reference layer stack in float64 (oracle/torch_ref.py on the device)."""
    from oracle import torch_ref as tr
    dev = _dev()
    B, C, T = 1024, 64, 512
    m = random_model(C, T, F1=16, D=4, p=0.25, seed=0, perturb_bn=False).to(dev).train()
    state = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    x_np, y_np = make_inputs(B, C, T, 4321)
    m2, m3 = make_masks(B, 64, T, 17, 0.25)
    x, y = torch.from_numpy(x_np).to(dev), torch.from_numpy(y_np).to(dev)
    masks = (torch.from_numpy(m2).to(dev), torch.from_numpy(m3).to(dev))
    m.set_dropout_masks(*masks)
    logits = m(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    ref = tr.TorchRefEEGNet(state, p=0.25, device=dev, dtype=torch.float64)
    rl = ref(x.double(), masks)
    rloss = torch.nn.functional.cross_entropy(rl, y)
    rloss.backward()
    assert_close(logits.detach().cpu().numpy(), rl.detach().cpu().numpy(), name="cfg5 B1024 logits")
    assert abs(float(loss) - float(rloss)) <= 1e-4 * max(1.0, abs(float(rloss)))
    assert_grads_close(grads_of(m), {k: ref.params[k].grad.cpu().numpy() for k in PARAM_NAMES},
                       prefix="cfg5 B1024 grad.")
    for k, b in m.named_buffers():
        r = ref.buffers[k].cpu().numpy()
        if "running_mean" in k:
            assert_close(b.cpu().numpy(), r, atol_abs=1e-6, name=k)
        elif "running_var" in k:
            assert_close(b.cpu().numpy(), r, name=k)


@pytest.mark.parametrize("C,T,F1,D,B", [(64, 512, 16, 4, 40), (22, 257, 16, 4, 33), (22, 256, 12, 2, 5),
                                        (40, 128, 12, 4, 7)])
def test_wide_eval_matches_oracle(C, T, F1, D, B):
    dev = _dev()
    m = random_model(C, T, F1=F1, D=D, seed=7 * C + T).to(dev).eval()
    x_np, _ = make_inputs(B, C, T, B + T)
    with torch.no_grad():
        out = m(torch.from_numpy(x_np).to(dev)).cpu().numpy()
    assert_close(out, oracle_eval(m, x_np), name=f"wide eval EEGNet-{F1},{D} {C}x{T}")
