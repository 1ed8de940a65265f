"""GPU parity of the bf16 batched eval forward (eegnet_forward_eval_bf16, SURVEY 8(f) row 4, BASELINE
cfg5: EEGNet-16,4 on 64ch x 512) against the float64 CPU oracle (oracle/numpy_ref.py, pinned to the
reference's golden vectors by tests/test_oracle.py) on the same bf16-rounded input.

Tolerance: |gpu - ref| <= 2e-2 * max|ref| elementwise.  The input is rounded to
bf16 before the oracle sees it, so the error budget covers only the kernel's own bf16 operands (ws,
w1, W3 and the intermediates s, z), each ~2^-9 relative, accumulated in fp32.  Predicted classes
must agree except where the oracle's top-2 margin is inside that tolerance.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import numpy_ref as nr

pytestmark = pytest.mark.gpu

TOL = 2e-2

# (C, T, F1, D, B): cfg5, the benchmark shape, the real-data T=257 (element staging), test shapes
CASES = [
    (64, 512, 16, 4, 48),      # BASELINE cfg5: EEGNet-16,4, 64ch x 512
    (22, 256, 8, 2, 37),       # cfg2 shape
    (22, 257, 8, 2, 5),        # T % 8 != 0: 2-byte staging path, pool floor truncation
    (64, 128, 8, 2, 9),        # reference test shape (64, 128)
    (32, 512, 8, 2, 3),        # reference test shape (32, 512)
    (8, 64, 8, 2, 1),          # reference test shape (8, 64), B = 1
    (40, 256, 12, 2, 7),       # F2 = 24 (rows padded to 32), C = 40 (two K-steps, padded)
]


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _model(C, T, F1, D, seed):
    from eegnetreplication_amd import EEGNet
    torch.manual_seed(seed)
    m = EEGNet(C, T, F1=F1, D=D, p=0.5)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        params = dict(m.named_parameters())
        for bn in ("temporal.1", "aggregation.0", "block_2.2"):
            params[bn + ".weight"].copy_(0.5 + torch.rand(params[bn + ".weight"].shape, generator=g))
            params[bn + ".bias"].copy_(0.2 * torch.randn(params[bn + ".bias"].shape, generator=g))
        for name, b in m.named_buffers():
            if name.endswith("running_mean"):
                b.copy_(0.1 * torch.randn(b.shape, generator=g))
            elif name.endswith("running_var"):
                b.copy_(0.3 + torch.rand(b.shape, generator=g))
    return m


def _oracle(m, x32: np.ndarray) -> np.ndarray:
    params = {k: p.detach().cpu().numpy() for k, p in m.named_parameters()}
    bufs = {k: b.detach().cpu().numpy() for k, b in m.named_buffers()}
    out, _, _ = nr.forward(params, bufs, x32, train=False)
    return np.asarray(out, dtype=np.float64)


def _check(out: np.ndarray, ref: np.ndarray, what: str):
    scale = float(np.abs(ref).max())
    err = np.abs(out - ref)
    assert np.all(np.isfinite(out)), f"{what}: non-finite logits"
    assert err.max() <= TOL * scale, f"{what}: max |err| {err.max():.3e} > {TOL} * {scale:.3e}"
    top2 = np.sort(ref, axis=1)[:, -2:]
    decided = (top2[:, 1] - top2[:, 0]) > 2 * TOL * scale
    assert np.array_equal(out.argmax(1)[decided], ref.argmax(1)[decided]), f"{what}: class flips"


@pytest.mark.parametrize("C,T,F1,D,B", CASES)
def test_bf16_eval_matches_oracle(C, T, F1, D, B):
    dev = _dev()
    m = _model(C, T, F1, D, seed=C * 1000 + T).to(dev).eval()
    rng = np.random.default_rng(C + T + B)
    xb = torch.from_numpy(rng.standard_normal((B, C, T)).astype(np.float32)).to(torch.bfloat16)
    with torch.no_grad():
        out = m(xb.to(dev)).cpu().numpy()
    ref = _oracle(m.cpu(), xb.float().numpy())
    _check(out, ref, f"bf16 eval C={C} T={T} F1={F1} D={D} B={B}")


def test_bf16_eval_agrees_with_fp32_kernel():
    """Same model, same (bf16-representable) input: the bf16 kernel against the fp32 HIP eval
    kernel on the cfg2 shape, where both exist."""
    dev = _dev()
    m = _model(22, 256, 8, 2, seed=7).to(dev).eval()
    x = torch.randn(256, 22, 256, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
    with torch.no_grad():
        out16 = m(x.to(dev)).cpu().numpy()
        out32 = m(x.float().to(dev)).cpu().numpy()
    _check(out16, out32.astype(np.float64), "bf16 vs fp32 kernel")


def test_bf16_eval_full_size_batch_invariance():
    """cfg5 at a full batch: every trial's logits are bit-identical to the same trial run alone
    (each trial is one workgroup's private computation, whatever its position or neighbours), and a
    sample of them matches the oracle."""
    dev = _dev()
    B = 8192
    m = _model(64, 512, 16, 4, seed=11).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(B, 64, 512, device=dev, generator=g).to(torch.bfloat16)
    with torch.no_grad():
        full = m(x)
        idx = torch.tensor([0, 1, 255, 256, 4097, B - 1], device=dev)
        part = m(x[idx].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(full[idx], part), "logits depend on the batch a trial is run in"
    assert torch.isfinite(full).all()
    ref = _oracle(m.cpu(), x[idx].float().cpu().numpy())
    _check(full[idx].cpu().numpy(), ref, "cfg5 B=8192 sample")


def test_bf16_eval_rejects_bad_input():
    dev = _dev()
    m = _model(22, 256, 8, 2, seed=1).to(dev).eval()
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 21, 256, dtype=torch.bfloat16, device=dev))
    m.train()
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 22, 256, dtype=torch.bfloat16, device=dev))


@pytest.mark.parametrize("C,T,F1,D,nwg", [(64, 512, 16, 4, 512), (22, 256, 8, 2, 256)])
def test_bf16_eval_nonfinite_trial_stays_private(C, T, F1, D, nwg):
    """A trial with non-finite input must not leak into the next trial a workgroup runs (in the
    reference every trial's output is its own, model.py:91-99).  The cfg5 chunk kernel lays the block-2
    tail's z image over the s rows whose pad positions the FIR reads with zero taps (0 * Inf = NaN),
    so those pads are re-zeroed after every tail.  The first trial of every workgroup is
    NaN / Inf; every later trial must come out finite and bit-identical to its run without them."""
    dev = _dev()
    m = _model(C, T, F1, D, seed=23).to(dev).eval()
    B = 3 * nwg                                        # grid = nwg workgroups: three trials each
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(B, C, T, device=dev, generator=g).to(torch.bfloat16)
    x[:nwg // 2] = float("nan")
    x[nwg // 2:nwg, :, T // 3] = float("inf")
    with torch.no_grad():
        full = m(x)
        clean = m(x[nwg:].contiguous())
    torch.cuda.synchronize()
    assert torch.isfinite(full[nwg:]).all(), "a non-finite trial leaked into a later trial"
    assert torch.equal(full[nwg:], clean), "later trials depend on the earlier trials of their workgroup"
