"""CPU oracle (TEST INFRASTRUCTURE ONLY): fp32 stock-PyTorch restatement of the reference step.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this.

The reference is 100 % Python on stock ATen ops; its model cannot travel to the GPU box,
so this file restates the identical layer stack with ``torch.nn.functional`` calls on CPU tensors:

* EEGNet.forward          /root/reference/src/eegnet_repl/model.py:91-99 (layers model.py:22-84)
* grad clamps             model.py:43-44, 83-84 (tensor hooks on the two weights)
* CrossEntropyLoss        train.py:103
* Adam(lr=1e-3,eps=1e-7)  train.py:94-101 (torch.optim.Adam itself, CPU single-tensor path)

It is the ``bench.py`` CPU baseline (``kind: "port"``): the same ATen kernels the reference runs on
CPU, timed on the GPU host's cores.  It is pinned to the reference by ``tests/test_oracle.py``
against the golden vectors in ``tests/golden``.  Dropout masks may be injected (``masks=(m2, m3)``)
so that results are comparable; with ``masks=None`` it draws them from torch's RNG like nn.Dropout.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .numpy_ref import BN_EPS, BN_MOMENTUM, PARAM_NAMES, BN_PREFIXES, same_pad


class TorchRefEEGNet:
    """Holds fp32 leaf tensors named like the reference state_dict; forward == model.py:91-99."""

    def __init__(self, state: dict, p: float = 0.5, device="cpu", dtype=torch.float32):
        """``dtype=torch.float64`` turns the same ATen layer stack into a float64 oracle (used by
        the GPU tests at sizes the numpy oracle is too slow for)."""
        self.p = p
        self.params = {k: torch.as_tensor(state[k], dtype=dtype, device=device)
                       .clone().requires_grad_(True) for k in PARAM_NAMES}
        self.buffers = {}
        for pre in BN_PREFIXES:
            for suf in ("running_mean", "running_var"):
                self.buffers[f"{pre}.{suf}"] = torch.as_tensor(
                    state[f"{pre}.{suf}"], dtype=dtype, device=device).clone()
            self.buffers[f"{pre}.num_batches_tracked"] = torch.as_tensor(
                state[f"{pre}.num_batches_tracked"], dtype=torch.int64, device=device).clone()
        # model.py:44 and model.py:84 -- clamp the gradient, not the weight
        self.params["spatial.weight"].register_hook(lambda g: torch.clamp(g, -1.0, 1.0))
        self.params["classifier.weight"].register_hook(lambda g: torch.clamp(g, -0.25, 0.25))
        self.training = True

    def parameters(self):
        return [self.params[k] for k in PARAM_NAMES]

    def _bn(self, pre, a):
        b = self.buffers
        if self.training:
            b[f"{pre}.num_batches_tracked"] += 1
        return F.batch_norm(a, b[f"{pre}.running_mean"], b[f"{pre}.running_var"],
                            self.params[f"{pre}.weight"], self.params[f"{pre}.bias"],
                            training=self.training, momentum=BN_MOMENTUM, eps=BN_EPS)

    def _drop(self, a, mask):
        if not self.training or self.p == 0.0:
            return a
        if mask is None:
            return F.dropout(a, self.p, training=True)
        return a * (mask.to(a.dtype) / (1.0 - self.p))

    def forward(self, x, masks=None):
        P = self.params
        F1 = P["temporal.0.weight"].shape[0]
        F2 = P["spatial.weight"].shape[0]
        K1 = P["temporal.0.weight"].shape[-1]
        m2 = m3 = None
        if masks is not None:
            m2 = torch.as_tensor(masks[0]).reshape(x.shape[0], F2, 1, -1)
            m3 = torch.as_tensor(masks[1]).reshape(x.shape[0], F2, 1, -1)
        a = x.unsqueeze(1)
        a = F.pad(a, same_pad(K1))
        a = F.conv2d(a, P["temporal.0.weight"])
        a = self._bn("temporal.1", a)
        a = F.conv2d(a, P["spatial.weight"], groups=F1)
        a = self._bn("aggregation.0", a)
        a = F.elu(a)
        a = F.avg_pool2d(a, (1, 4))
        a = self._drop(a, m2)
        a = F.conv2d(F.pad(a, same_pad(16)), P["block_2.0.weight"], groups=F2)
        a = F.conv2d(a, P["block_2.1.weight"])
        a = self._bn("block_2.2", a)
        a = F.elu(a)
        a = F.avg_pool2d(a, (1, 8))
        a = self._drop(a, m3)
        a = a.flatten(1)
        return F.linear(a, P["classifier.weight"], P["classifier.bias"])

    __call__ = forward


def init_state(C: int, T: int, F1: int = 8, D: int = 2, K1: int = 32) -> dict:
    """The reference's initial state_dict: its modules constructed in model.py:22-84's order with
    torch.nn defaults (kaiming-uniform conv / linear weights, uniform linear bias, BN gamma 1, beta 0,
    running 0 / 1), drawing from torch's global generator exactly as EEGNet() does -- so
    ``torch.manual_seed(s); init_state(...)`` equals the reference's (and the product's) EEGNet(...)
    state after the same seed, without importing either (tools/accuracy_parity.py reference workers).
    Only the modules with parameters draw; ELU / pool / dropout / flatten draw nothing."""
    import torch.nn as nn
    F2 = F1 * D
    mods = [("temporal.0", nn.Conv2d(1, F1, kernel_size=(1, K1), padding="same", bias=False)),
            ("temporal.1", nn.BatchNorm2d(F1)),
            ("spatial", nn.Conv2d(F1, F2, kernel_size=(C, 1), padding="valid", groups=F1, bias=False)),
            ("aggregation.0", nn.BatchNorm2d(F2)),
            ("block_2.0", nn.Conv2d(F2, F2, kernel_size=(1, 16), padding="same", groups=F2, bias=False)),
            ("block_2.1", nn.Conv2d(F2, F2, kernel_size=(1, 1), padding="same", bias=False)),
            ("block_2.2", nn.BatchNorm2d(F2)),
            ("classifier", nn.Linear(F2 * (T // 32), 4, bias=True))]
    state = {}
    for pre, m in mods:
        for k, v in m.state_dict().items():
            state[f"{pre}.{k}"] = v.detach().clone()
    return state


def make_optimizer(model: TorchRefEEGNet, lr=1e-3, eps=1e-7):
    return torch.optim.Adam(model.parameters(), lr=lr, eps=eps, foreach=None, fused=None)


def train_step(model: TorchRefEEGNet, opt, x, y, masks=None):
    """model.py:141-148: forward, CE, zero_grad, backward, step.  Returns the loss tensor."""
    logits = model(x, masks)
    loss = F.cross_entropy(logits, y)
    opt.zero_grad()
    loss.backward()
    opt.step()
    return loss, logits
