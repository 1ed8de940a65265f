"""CPU oracle (TEST INFRASTRUCTURE ONLY): float64 numpy restatement of the reference EEGNet step.

This module is the checker, never the product.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product path (``eegnetreplication_amd``)
never imports anything under ``oracle/``.

It restates, layer by layer and in float64, what the reference computes through stock ATen ops:

* model       -- /root/reference/src/eegnet_repl/model.py:12-99  (``EEGNet.__init__`` / ``forward``)
* grad clamps -- model.py:43-44 (spatial, +-1.0) and model.py:83-84 (classifier, +-0.25); they clamp
                 the *gradient* (tensor hooks), not the weights
* loss        -- train.py:103 ``nn.CrossEntropyLoss()`` (mean over the batch), called at model.py:142
* optimizer   -- train.py:94-101 ``optim.Adam(lr=1e-3, eps=1e-7)``; math of torch/optim/adam.py:457,476,
                 531-547 (single-tensor path)
* BN          -- torch.nn.BatchNorm2d defaults (eps=1e-5, momentum=0.1, biased batch var for the
                 normalisation, unbiased var n/(n-1) for ``running_var``; model.py:32,47,71)

Parity is pinned by golden vectors produced by the reference itself
(``tests/golden/make_golden.py``, run in the survey container where ``/root/reference`` imports);
``tests/test_oracle.py`` checks this module against every one of them.

Dropout masks cannot be reproduced from torch's CPU RNG stream, so they are *injected*: ``masks`` is
``(m2, m3)`` with shapes ``[B,F2,T1]`` and ``[B,F2,T2]`` (1 = keep).  ``p == 0`` needs no masks.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
K2 = 16          # model.py:57   block_2 depthwise kernel (1,16)
POOL1 = 4        # model.py:49   AvgPool2d((1,4))
POOL2 = 8        # model.py:73   AvgPool2d((1,8))
N_CLASSES = 4    # model.py:80
SPATIAL_CLAMP = 1.0      # model.py:43
CLASSIFIER_CLAMP = 0.25  # model.py:83

PARAM_NAMES = (
    "temporal.0.weight", "temporal.1.weight", "temporal.1.bias", "spatial.weight",
    "aggregation.0.weight", "aggregation.0.bias", "block_2.0.weight", "block_2.1.weight",
    "block_2.2.weight", "block_2.2.bias", "classifier.weight", "classifier.bias",
)
BN_PREFIXES = ("temporal.1", "aggregation.0", "block_2.2")


@dataclass(frozen=True)
class Dims:
    C: int
    T: int
    F1: int = 8
    D: int = 2
    K1: int = 32

    @property
    def F2(self) -> int:
        return self.F1 * self.D

    @property
    def T1(self) -> int:
        return self.T // POOL1

    @property
    def T2(self) -> int:
        return self.T1 // POOL2

    @property
    def n_feat(self) -> int:
        # model.py:79 uses F2*(T//32); floor(floor(T/4)/8) == floor(T/32)
        return self.F2 * (self.T // 32)


def same_pad(k: int) -> tuple[int, int]:
    """torch 'same' padding for an even kernel: left (k-1)//2, right the rest."""
    left = (k - 1) // 2
    return left, k - 1 - left


def _pad_t(a: np.ndarray, k: int) -> np.ndarray:
    left, right = same_pad(k)
    pad = [(0, 0)] * (a.ndim - 1) + [(left, right)]
    return np.pad(a, pad)


def _corr_same(a: np.ndarray, w: np.ndarray) -> np.ndarray:
    """out[..., t] = sum_k w[..., k] * apad[..., t+k]; w broadcasts against a's leading dims."""
    k = w.shape[-1]
    ap = _pad_t(a, k)
    T = a.shape[-1]
    out = np.zeros(np.broadcast_shapes(a.shape, w.shape[:-1] + (T,)), dtype=np.float64)
    for j in range(k):
        out += w[..., j:j + 1] * ap[..., j:j + T]
    return out


def _corr_same_wgrad(dout: np.ndarray, a: np.ndarray, k: int, axes: tuple[int, ...]) -> np.ndarray:
    """dw[..., j] = sum_{axes} dout[..., t] * apad[..., t+j]."""
    ap = _pad_t(a, k)
    T = a.shape[-1]
    cols = [np.sum(dout * ap[..., j:j + T], axis=axes) for j in range(k)]
    return np.stack(cols, axis=-1)


def _corr_same_dgrad(dout: np.ndarray, w: np.ndarray) -> np.ndarray:
    """Adjoint of _corr_same with respect to its input a."""
    k = w.shape[-1]
    left, _ = same_pad(k)
    T = dout.shape[-1]
    dap = np.zeros(dout.shape[:-1] + (T + k - 1,), dtype=np.float64)
    for j in range(k):
        dap[..., j:j + T] += w[..., j:j + 1] * dout
    return dap[..., left:left + T]


def _elu(z):
    # nn.ELU(alpha=1): x if x > 0 else expm1(x)   (model.py:48,72)
    return np.where(z > 0, z, np.expm1(np.minimum(z, 0.0)))


def _elu_grad(z):
    return np.where(z > 0, 1.0, np.exp(np.minimum(z, 0.0)))


def _avgpool(a: np.ndarray, k: int) -> np.ndarray:
    n = a.shape[-1] // k          # floor truncation (T=257 drops the last sample)
    return a[..., :n * k].reshape(a.shape[:-1] + (n, k)).mean(axis=-1)


def _avgpool_bwd(dout: np.ndarray, k: int, length: int) -> np.ndarray:
    n = dout.shape[-1]
    d = np.zeros(dout.shape[:-1] + (length,), dtype=np.float64)
    d[..., :n * k] = np.repeat(dout / k, k, axis=-1)
    return d


def _bn_train(a: np.ndarray, axes: tuple[int, ...], gamma, beta, shape):
    n = int(np.prod([a.shape[i] for i in axes]))
    mu = a.mean(axis=axes)
    var = a.var(axis=axes)                          # biased, used for normalisation
    invstd = 1.0 / np.sqrt(var + BN_EPS)
    xh = (a - mu.reshape(shape)) * invstd.reshape(shape)
    y = xh * gamma.reshape(shape) + beta.reshape(shape)
    return y, xh, mu, var, invstd, n


def _bn_eval(a, rm, rv, gamma, beta, shape):
    invstd = 1.0 / np.sqrt(rv + BN_EPS)
    return (a - rm.reshape(shape)) * (invstd * gamma).reshape(shape) + beta.reshape(shape)


def _bn_bwd(dy, xh, invstd, gamma, axes, shape):
    n = int(np.prod([dy.shape[i] for i in axes]))
    dbeta = dy.sum(axis=axes)
    dgamma = (dy * xh).sum(axis=axes)
    dx = (gamma * invstd).reshape(shape) * (
        dy - (dbeta / n).reshape(shape) - xh * (dgamma / n).reshape(shape))
    return dx, dgamma, dbeta


def dims_from_params(params: dict, C: int, T: int) -> Dims:
    F1 = params["temporal.0.weight"].shape[0]
    K1 = params["temporal.0.weight"].shape[-1]
    F2 = params["spatial.weight"].shape[0]
    return Dims(C=C, T=T, F1=F1, D=F2 // F1, K1=K1)


def forward(params: dict, buffers: dict, x: np.ndarray, *, train: bool, p: float = 0.0,
            masks=None):
    """EEGNet.forward (model.py:91-99).  Returns (logits, cache, new_buffers).

    ``buffers`` holds ``<bn>.running_mean/.running_var/.num_batches_tracked`` for the three BNs;
    in train mode the returned copy carries the momentum update (torch BatchNorm2d semantics).
    """
    x = np.asarray(x, dtype=np.float64)
    B, C, T = x.shape
    dm = dims_from_params(params, C, T)
    F1, D, F2 = dm.F1, dm.D, dm.F2
    P = {k: np.asarray(v, dtype=np.float64) for k, v in params.items()}
    nb = {k: np.array(v, copy=True) for k, v in buffers.items()}
    drop = train and p > 0.0
    if drop:
        if masks is None:
            raise ValueError("train-mode dropout needs injected masks (m2, m3)")
        m2 = np.asarray(masks[0], dtype=np.float64)
        m3 = np.asarray(masks[1], dtype=np.float64)
        scale = 1.0 / (1.0 - p) if p < 1.0 else 0.0

    # temporal conv (model.py:23-30): u[b,g,c,t] = sum_k w1[g,k] xpad[b,c,t+k]
    w1 = P["temporal.0.weight"].reshape(F1, dm.K1)
    u = _corr_same(x[:, None, :, :], w1[None, :, None, :])           # [B,F1,C,T]

    def bn(name, a, axes, shape):
        g, bta = P[name + ".weight"], P[name + ".bias"]
        if train:
            y, xh, mu, var, invstd, n = _bn_train(a, axes, g, bta, shape)
            rm, rv = nb[name + ".running_mean"], nb[name + ".running_var"]
            nb[name + ".running_mean"] = ((1 - BN_MOMENTUM) * rm + BN_MOMENTUM * mu).astype(rm.dtype)
            nb[name + ".running_var"] = ((1 - BN_MOMENTUM) * rv
                                         + BN_MOMENTUM * var * n / (n - 1)).astype(rv.dtype)
            nb[name + ".num_batches_tracked"] = nb[name + ".num_batches_tracked"] + 1
            return y, xh, invstd
        y = _bn_eval(a, nb[name + ".running_mean"].astype(np.float64),
                     nb[name + ".running_var"].astype(np.float64), g, bta, shape)
        return y, None, None

    y1, xh1, inv1 = bn("temporal.1", u, (0, 2, 3), (1, F1, 1, 1))     # model.py:32
    # spatial depthwise conv (model.py:34-41): y2[b,o,t] = sum_c ws[o,c] y1[b,o//D,c,t]
    ws = P["spatial.weight"].reshape(F2, C)
    grp = np.arange(F2) // D
    y2 = np.einsum("oc,boct->bot", ws, y1[:, grp, :, :])
    z2, xh2, inv2 = bn("aggregation.0", y2, (0, 2), (1, F2, 1))        # model.py:47
    e2 = _elu(z2)
    p2 = _avgpool(e2, POOL1)                                           # [B,F2,T1]
    d2 = p2 * m2 * scale if drop else p2
    # separable block (model.py:54-69)
    w2 = P["block_2.0.weight"].reshape(F2, K2)
    q = _corr_same(d2, w2[None, :, :])
    W3 = P["block_2.1.weight"].reshape(F2, F2)
    r = np.einsum("ji,bit->bjt", W3, q)
    z3, xh3, inv3 = bn("block_2.2", r, (0, 2), (1, F2, 1))             # model.py:71
    e3 = _elu(z3)
    p3 = _avgpool(e3, POOL2)                                           # [B,F2,T2]
    d3 = p3 * m3 * scale if drop else p3
    h = d3.reshape(B, -1)                                              # Flatten (model.py:75)
    Wfc = P["classifier.weight"]
    logits = h @ Wfc.T + P["classifier.bias"]                          # model.py:78-82
    cache = dict(x=x, dims=dm, P=P, u=u, xh1=xh1, inv1=inv1, y1=y1, grp=grp, z2=z2, xh2=xh2,
                 inv2=inv2, d2=d2, q=q, z3=z3, xh3=xh3, inv3=inv3, h=h, drop=drop,
                 m2=m2 if drop else None, m3=m3 if drop else None,
                 scale=scale if drop else 1.0)
    return logits, cache, nb


def cross_entropy(logits: np.ndarray, labels: np.ndarray):
    """nn.CrossEntropyLoss() mean reduction (train.py:103).  Returns (loss, dlogits)."""
    z = np.asarray(logits, dtype=np.float64)
    B = z.shape[0]
    zmax = z.max(axis=1, keepdims=True)
    lse = zmax[:, 0] + np.log(np.exp(z - zmax).sum(axis=1))
    loss = float(np.mean(lse - z[np.arange(B), labels]))
    sm = np.exp(z - lse[:, None])
    dz = sm.copy()
    dz[np.arange(B), labels] -= 1.0
    return loss, dz / B


def backward(cache: dict, dlogits: np.ndarray, clamp: bool = True) -> dict:
    """loss.backward() through EEGNet, including the two gradient clamps (model.py:44,84);
    ``clamp=False`` returns the raw gradients (the scale the clamp is applied at).

    Returns grads keyed by parameter name, shaped like the parameters.
    """
    dm: Dims = cache["dims"]
    P = cache["P"]
    B, C, T = cache["x"].shape
    F1, D, F2, K1 = dm.F1, dm.D, dm.F2, dm.K1
    dz = np.asarray(dlogits, dtype=np.float64)
    g = {}
    h = cache["h"]
    g["classifier.weight"] = np.clip(dz.T @ h, -CLASSIFIER_CLAMP, CLASSIFIER_CLAMP) if clamp else dz.T @ h
    g["classifier.bias"] = dz.sum(axis=0)
    dh = dz @ P["classifier.weight"]
    dd3 = dh.reshape(B, F2, dm.T2)
    dp3 = dd3 * cache["m3"] * cache["scale"] if cache["drop"] else dd3
    de3 = _avgpool_bwd(dp3, POOL2, dm.T1)
    dz3 = de3 * _elu_grad(cache["z3"])
    dr, g["block_2.2.weight"], g["block_2.2.bias"] = _bn_bwd(
        dz3, cache["xh3"], cache["inv3"], P["block_2.2.weight"], (0, 2), (1, F2, 1))
    q = cache["q"]
    W3 = P["block_2.1.weight"].reshape(F2, F2)
    g["block_2.1.weight"] = np.einsum("bjt,bit->ji", dr, q).reshape(F2, F2, 1, 1)
    dq = np.einsum("ji,bjt->bit", W3, dr)
    w2 = P["block_2.0.weight"].reshape(F2, K2)
    g["block_2.0.weight"] = _corr_same_wgrad(dq, cache["d2"], K2, (0, 2)).reshape(F2, 1, 1, K2)
    dd2 = _corr_same_dgrad(dq, w2[None, :, :])
    dp2 = dd2 * cache["m2"] * cache["scale"] if cache["drop"] else dd2
    de2 = _avgpool_bwd(dp2, POOL1, T)
    dz2 = de2 * _elu_grad(cache["z2"])
    dy2, g["aggregation.0.weight"], g["aggregation.0.bias"] = _bn_bwd(
        dz2, cache["xh2"], cache["inv2"], P["aggregation.0.weight"], (0, 2), (1, F2, 1))
    y1 = cache["y1"]
    grp = cache["grp"]
    dws = np.einsum("bot,boct->oc", dy2, y1[:, grp, :, :])
    g["spatial.weight"] = (np.clip(dws, -SPATIAL_CLAMP, SPATIAL_CLAMP) if clamp else dws).reshape(F2, 1, C, 1)
    ws = P["spatial.weight"].reshape(F2, C)
    dy1 = np.zeros((B, F1, C, T))
    for o in range(F2):
        dy1[:, o // D] += ws[o][None, :, None] * dy2[:, o, None, :]
    du, g["temporal.1.weight"], g["temporal.1.bias"] = _bn_bwd(
        dy1, cache["xh1"], cache["inv1"], P["temporal.1.weight"], (0, 2, 3), (1, F1, 1, 1))
    dW1 = _corr_same_wgrad(du, cache["x"][:, None, :, :], K1, (0, 2, 3))
    g["temporal.0.weight"] = dW1.reshape(F1, 1, 1, K1)
    return g


@dataclass
class AdamState:
    step: int
    m: dict
    v: dict


def adam_init(params: dict) -> AdamState:
    return AdamState(0, {k: np.zeros_like(v, dtype=np.float64) for k, v in params.items()},
                     {k: np.zeros_like(v, dtype=np.float64) for k, v in params.items()})


def adam_step(params: dict, grads: dict, st: AdamState, lr=1e-3, betas=(0.9, 0.999), eps=1e-7):
    """torch Adam, weight_decay=0, amsgrad=False (torch/optim/adam.py:457,476,531-547)."""
    b1, b2 = betas
    st.step += 1
    bc1 = 1.0 - b1 ** st.step
    bc2 = 1.0 - b2 ** st.step
    out = {}
    for k, p in params.items():
        gk = np.asarray(grads[k], dtype=np.float64)
        st.m[k] = st.m[k] + (1.0 - b1) * (gk - st.m[k])          # exp_avg.lerp_(grad, 1-beta1)
        st.v[k] = b2 * st.v[k] + (1.0 - b2) * gk * gk             # mul_(b2).addcmul_(g,g,1-b2)
        denom = np.sqrt(st.v[k]) / math.sqrt(bc2) + eps
        out[k] = np.asarray(p, dtype=np.float64) - (lr / bc1) * st.m[k] / denom
    return out


def train_step(params, buffers, x, labels, st: AdamState, *, p=0.0, masks=None, lr=1e-3,
               eps=1e-7):
    """One hot-loop iteration of model.py:136-148: forward, CE, backward (+clamps), Adam."""
    logits, cache, nb = forward(params, buffers, x, train=True, p=p, masks=masks)
    loss, dl = cross_entropy(logits, labels)
    grads = backward(cache, dl)
    newp = adam_step(params, grads, st, lr=lr, eps=eps)
    return dict(logits=logits, loss=loss, grads=grads, params=newp, buffers=nb)
