"""Test-side helpers shared by the GPU parity tests: random EEGNet instances with non-trivial BN
state, the float64 oracle step with injected masks, and a numpy restatement of the on-device
dropout generator (eegnet_common.h keep_mul / eegnet_host.hip mix_key + set_key)."""

from __future__ import annotations

import numpy as np
import torch

from golden_util import PARAM_NAMES
from oracle import numpy_ref as nr

M64 = (1 << 64) - 1


def mix_key(seed: int, offset: int) -> int:
    """splitmix64 finalizer of (seed, offset) -- eegnet_host.hip mix_key."""
    z = (seed * 0xD1B54A32D192ED03 + offset * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _keep(n: int, key: int, pthr: int) -> np.ndarray:
    h = np.arange(n, dtype=np.uint64).astype(np.uint32)
    h = h * np.uint32(0x9E3779B1) + np.uint32(key)
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x85EBCA6B)
    h ^= h >> np.uint32(13)
    h *= np.uint32(0xC2B2AE35)
    h ^= h >> np.uint32(16)
    return ((h >> np.uint32(8)) >= np.uint32(pthr)).astype(np.uint8)


def device_masks(B: int, F2: int, T: int, seed: int, offset: int, p: float):
    """The keep-masks the on-device generator draws for (seed, offset): [B,F2,T//4], [B,F2,T//128]
    (flat indices (b*F2+o)*T1+q and b*F2*T2 + o*T2 + t, per-layer 32-bit keys)."""
    key = mix_key(seed, offset)
    k0 = key & 0xFFFFFFFF
    k1 = ((key >> 32) ^ 0x5BD1E995) & 0xFFFFFFFF
    pthr = int(min(16777216.0, max(0.0, float(np.float32(p)) * 16777216.0)))
    T1 = T // 4
    T2 = T1 // 8
    m2 = _keep(B * F2 * T1, k0, pthr).reshape(B, F2, T1)
    m3 = _keep(B * F2 * T2, k1, pthr).reshape(B, F2, T2)
    return m2, m3


def random_model(C, T, F1=8, D=2, K1=32, p=0.5, seed=0, perturb_bn=True):
    """EEGNet with default init, then BN affine parameters and running statistics moved off their
    identity values so every BN term is exercised."""
    from eegnetreplication_amd import EEGNet
    torch.manual_seed(seed)
    m = EEGNet(C, T, F1=F1, D=D, p=p, K1=K1)
    if perturb_bn:
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


def state_np(m):
    params = {k: p.detach().cpu().numpy() for k, p in m.named_parameters()}
    bufs = {k: b.detach().cpu().numpy() for k, b in m.named_buffers()}
    return params, bufs


def oracle_step(m, x, y, p=0.0, masks=None, loss_scale=1.0):
    """float64 oracle: logits, loss, clamped grads and updated buffers of one train-mode step."""
    params, bufs = state_np(m)
    logits, cache, nb = nr.forward(params, bufs, x, train=True, p=p, masks=masks)
    loss, dl = nr.cross_entropy(logits, y)
    grads = nr.backward(cache, dl * loss_scale)
    return logits, loss, grads, nb, dl


def oracle_eval(m, x):
    params, bufs = state_np(m)
    logits, _, _ = nr.forward(params, bufs, x, train=False)
    return logits


def grads_of(model):
    return {k: p.grad.detach().cpu().numpy() for k, p in model.named_parameters()}


def flat_to_dict(model, flat):
    out, o = {}, 0
    for k, p in model.named_parameters():
        out[k] = flat[o:o + p.numel()].view(p.shape).detach().cpu().numpy()
        o += p.numel()
    return out


__all__ = ["PARAM_NAMES", "device_masks", "random_model", "oracle_step", "oracle_eval",
           "grads_of", "flat_to_dict", "state_np", "mix_key"]
