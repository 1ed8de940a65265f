"""float64 numpy model of the HIP kernels' *restructured* algorithm (design check, test-only).

The HIP path does not compute the reference's [B,F1,C,T] temporal-conv tensor.  It uses linearity:
  * spatial first: s[o] = sum_c ws[o,c] x[c];  v[o] = w1[g(o)] (*) s[o]  (== spatial(conv1(x)) / a1)
  * BN1 statistics from the lag-Gram of x (G[k,k'] = sum xpad[t+k] xpad[t+k']) and window sums
  * BN2 statistics from sum v, sum v^2 (y2 = a1 v + c1 W)
  * all backward weight-gradient reductions written as per-trial partial sums combined at the end
This file mirrors the kernel passes A..E and the five finalize steps one to one so the math can be
checked against ``oracle/numpy_ref.py`` on CPU before (and independently of) the GPU.
"""

from __future__ import annotations

import numpy as np

EPS = 1e-5
MOM = 0.1


def pad_row(a, K):
    P = (K - 1) // 2
    return np.pad(a, [(0, 0)] * (a.ndim - 1) + [(P, K - 1 - P)])


def step(params, buffers, x, labels=None, dlogits=None, *, p=0.0, masks=None):
    x = np.asarray(x, np.float64)
    B, C, T = x.shape
    w1 = params["temporal.0.weight"].reshape(-1, params["temporal.0.weight"].shape[-1]).astype(np.float64)
    F1, K1 = w1.shape
    ws = params["spatial.weight"].reshape(-1, C).astype(np.float64)
    F2 = ws.shape[0]
    D = F2 // F1
    grp = np.arange(F2) // D
    P = (K1 - 1) // 2
    T1, T2 = T // 4, T // 4 // 8
    g1, b1 = params["temporal.1.weight"].astype(np.float64), params["temporal.1.bias"].astype(np.float64)
    g2, b2 = params["aggregation.0.weight"].astype(np.float64), params["aggregation.0.bias"].astype(np.float64)
    g3, b3 = params["block_2.2.weight"].astype(np.float64), params["block_2.2.bias"].astype(np.float64)
    w2 = params["block_2.0.weight"].reshape(F2, 16).astype(np.float64)
    W3 = params["block_2.1.weight"].reshape(F2, F2).astype(np.float64)
    Wfc = params["classifier.weight"].astype(np.float64)
    bfc = params["classifier.bias"].astype(np.float64)
    sc = 1.0 / (1.0 - p) if p > 0 else 1.0
    m2 = masks[0].astype(np.float64) * sc if p > 0 else np.ones((B, F2, T1))
    m3 = masks[1].astype(np.float64) * sc if p > 0 else np.ones((B, F2, T2))
    out = {}

    # ---------------- pass A: per-trial partials ----------------
    X = pad_row(x, K1)                                 # [B,C,T+K1-1]
    G0 = np.zeros(K1)
    Ed = np.zeros((K1, K1))
    S0 = 0.0
    e1 = np.zeros(K1)
    for d in range(K1):
        G0[d] = np.sum(X[:, :, 0:T] * X[:, :, d:d + T])
        for j in range(K1 - 1 - d):
            Ed[d, j] = np.sum(X[:, :, T + j] * X[:, :, T + j + d] - X[:, :, j] * X[:, :, j + d])
    S0 = np.sum(X[:, :, 0:T])
    for j in range(K1 - 1):
        e1[j] = np.sum(X[:, :, T + j] - X[:, :, j])
    s = np.einsum("oc,bct->bot", ws, x)
    Sp = pad_row(s, K1)
    v = np.zeros((B, F2, T))
    for k in range(K1):
        v += w1[grp, k][None, :, None] * Sp[:, :, k:k + T]
    Sv, Sv2 = v.sum(axis=(0, 2)), (v * v).sum(axis=(0, 2))

    # ---------------- finalize 1 ----------------
    G = np.zeros((K1, K1))
    for d in range(K1):
        acc = G0[d]
        for k in range(K1 - d):
            G[k, k + d] = G[k + d, k] = acc
            if k < K1 - 1 - d:
                acc += Ed[d, k]
    S1 = np.zeros(K1)
    acc = S0
    for k in range(K1):
        S1[k] = acc
        if k < K1 - 1:
            acc += e1[k]
    n1 = B * C * T
    mu1 = w1 @ S1 / n1
    var1 = np.einsum("gk,kl,gl->g", w1, G, w1) / n1 - mu1 ** 2
    inv1 = 1.0 / np.sqrt(var1 + EPS)
    a1 = g1 * inv1
    c1 = b1 - a1 * mu1
    W = ws.sum(axis=1)
    n2 = B * T
    mv = Sv / n2
    varv = Sv2 / n2 - mv ** 2
    mu2 = a1[grp] * mv + c1[grp] * W
    var2 = a1[grp] ** 2 * varv
    inv2 = 1.0 / np.sqrt(var2 + EPS)
    alpha2 = a1[grp] * inv2
    beta2h = -alpha2 * mv
    nb = {k: np.array(v_, dtype=np.float64) for k, v_ in buffers.items()}
    nb["temporal.1.running_mean"] = (1 - MOM) * nb["temporal.1.running_mean"] + MOM * mu1
    nb["temporal.1.running_var"] = (1 - MOM) * nb["temporal.1.running_var"] + MOM * var1 * n1 / (n1 - 1)
    nb["aggregation.0.running_mean"] = (1 - MOM) * nb["aggregation.0.running_mean"] + MOM * mu2
    nb["aggregation.0.running_var"] = (1 - MOM) * nb["aggregation.0.running_var"] + MOM * var2 * n2 / (n2 - 1)

    # ---------------- pass B ----------------
    xh2 = alpha2[None, :, None] * v + beta2h[None, :, None]
    z2 = g2[None, :, None] * xh2 + b2[None, :, None]
    e2 = np.where(z2 > 0, z2, np.expm1(np.minimum(z2, 0)))
    de = np.where(z2 > 0, 1.0, np.exp(np.minimum(z2, 0)))
    p2 = e2[:, :, :4 * T1].reshape(B, F2, T1, 4).mean(-1)
    E1 = de[:, :, :4 * T1].reshape(B, F2, T1, 4).sum(-1)
    E2 = (de * xh2)[:, :, :4 * T1].reshape(B, F2, T1, 4).sum(-1)
    d2 = p2 * m2
    D2p = pad_row(d2, 16)
    q = np.zeros((B, F2, T1))
    for k in range(16):
        q += w2[None, :, k, None] * D2p[:, :, k:k + T1]
    r = np.einsum("ji,bit->bjt", W3, q)
    n3 = B * T1
    mu3, var3 = r.mean(axis=(0, 2)), r.var(axis=(0, 2))
    inv3 = 1.0 / np.sqrt(var3 + EPS)
    nb["block_2.2.running_mean"] = (1 - MOM) * nb["block_2.2.running_mean"] + MOM * mu3
    nb["block_2.2.running_var"] = (1 - MOM) * nb["block_2.2.running_var"] + MOM * var3 * n3 / (n3 - 1)
    for pre in ("temporal.1", "aggregation.0", "block_2.2"):
        nb[pre + ".num_batches_tracked"] = nb[pre + ".num_batches_tracked"] + 1
    out["buffers"] = nb

    # ---------------- pass C ----------------
    xh3 = (r - mu3[None, :, None]) * inv3[None, :, None]
    z3 = g3[None, :, None] * xh3 + b3[None, :, None]
    e3 = np.where(z3 > 0, z3, np.expm1(np.minimum(z3, 0)))
    de3f = np.where(z3 > 0, 1.0, np.exp(np.minimum(z3, 0)))
    p3 = e3[:, :, :8 * T2].reshape(B, F2, T2, 8).mean(-1)
    h = (p3 * m3).reshape(B, -1)
    logits = h @ Wfc.T + bfc
    out["logits"] = logits
    if dlogits is None:
        zmax = logits.max(1, keepdims=True)
        lse = zmax[:, 0] + np.log(np.exp(logits - zmax).sum(1))
        out["loss"] = float(np.mean(lse - logits[np.arange(B), labels]))
        dl = np.exp(logits - lse[:, None])
        dl[np.arange(B), labels] -= 1
        dl /= B
    else:
        dl = np.asarray(dlogits, np.float64)
    gr = {}
    gr["classifier.weight"] = np.clip(dl.T @ h, -0.25, 0.25)
    gr["classifier.bias"] = dl.sum(0)
    dp3 = (dl @ Wfc).reshape(B, F2, T2) * m3
    de3 = np.zeros((B, F2, T1))
    de3[:, :, :8 * T2] = np.repeat(dp3 / 8, 8, axis=-1)
    dz3 = de3 * de3f
    Sdz3, Sdz3x = dz3.sum(axis=(0, 2)), (dz3 * xh3).sum(axis=(0, 2))
    gr["block_2.2.weight"], gr["block_2.2.bias"] = Sdz3x, Sdz3

    # ---------------- pass D ----------------
    A3 = g3 * inv3
    dr = A3[None, :, None] * (dz3 - (Sdz3 / n3)[None, :, None] - xh3 * (Sdz3x / n3)[None, :, None])
    gr["block_2.1.weight"] = np.einsum("bjt,bit->ji", dr, q).reshape(F2, F2, 1, 1)
    dq = np.einsum("ji,bjt->bit", W3, dr)
    gr["block_2.0.weight"] = np.stack([np.sum(dq * D2p[:, :, k:k + T1], axis=(0, 2))
                                       for k in range(16)], -1).reshape(F2, 1, 1, 16)
    dqp = np.pad(dq, [(0, 0), (0, 0), (8, 7)])        # adjoint of pad (7 left, 8 right)
    dd2 = np.zeros((B, F2, T1))
    for k in range(16):
        dd2 += w2[None, :, k, None] * dqp[:, :, 15 - k:15 - k + T1]
    dp2 = dd2 * m2
    Sdz2 = np.sum(dp2 / 4 * E1, axis=(0, 2))
    Sdz2x = np.sum(dp2 / 4 * E2, axis=(0, 2))
    gr["aggregation.0.weight"], gr["aggregation.0.bias"] = Sdz2x, Sdz2

    # ---------------- pass E ----------------
    A2 = g2 * inv2
    Bo = -A2 * Sdz2 / n2
    Co = -A2 * Sdz2x / n2
    dz2 = np.zeros((B, F2, T))
    dz2[:, :, :4 * T1] = np.repeat(dp2 / 4, 4, axis=-1) * de[:, :, :4 * T1]
    dy2 = A2[None, :, None] * dz2 + Bo[None, :, None] + Co[None, :, None] * xh2
    Sdy, Sdyv = dy2.sum(axis=(0, 2)), (dy2 * v).sum(axis=(0, 2))
    Q = np.stack([np.sum(dy2 * Sp[:, :, k:k + T], axis=(0, 2)) for k in range(K1)], -1)   # [F2,K1]
    # e[o][j] = sum_k w1[g][k] dy2[o][j-k], only j in [P, P+T) is needed
    dyp = np.pad(dy2, [(0, 0), (0, 0), (K1 - 1, K1 - 1)])
    e = np.zeros((B, F2, T))
    for k in range(K1):
        # j = P + s ; dy2 index j - k = P + s - k -> padded index P + s - k + K1 - 1
        e += w1[grp, k][None, :, None] * dyp[:, :, P - k + K1 - 1:P - k + K1 - 1 + T]
    Xm = np.einsum("bct,bot->oc", x, e)

    # ---------------- finalize 5 ----------------
    dws = a1[grp, None] * Xm + c1[grp, None] * Sdy[:, None]
    gr["spatial.weight"] = np.clip(dws, -1, 1).reshape(F2, 1, C, 1)
    db1 = np.array([np.sum(W[grp == g] * Sdy[grp == g]) for g in range(F1)])
    dyu = np.array([np.sum(Sdyv[grp == g]) for g in range(F1)])
    dg1 = inv1 * (dyu - mu1 * db1)
    gr["temporal.1.weight"], gr["temporal.1.bias"] = dg1, db1
    Qg = np.stack([Q[grp == g].sum(0) for g in range(F1)])             # [F1,K1]
    uX = w1 @ G                                                        # [F1,K1]
    xhX = inv1[:, None] * (uX - mu1[:, None] * S1[None, :])
    dW1 = a1[:, None] * (Qg - (db1 / n1)[:, None] * S1[None, :] - (dg1 / n1)[:, None] * xhX)
    gr["temporal.0.weight"] = dW1.reshape(F1, 1, 1, K1)
    out["grads"] = gr
    return out
