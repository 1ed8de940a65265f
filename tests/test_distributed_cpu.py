"""Multi-process orchestration on CPU (gloo, world_size 2): the data-parallel step's
all-reduce -> clamp -> Adam order, and fold sharding / result gathering.  The HIP local step is
replaced by the CPU oracle (test-only stand-in); everything else is the product code."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_util import Golden, PARAM_NAMES


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat(d):
    return torch.cat([torch.as_tensor(np.asarray(d[k]), dtype=torch.float64).reshape(-1)
                      for k in PARAM_NAMES])


def _oracle_local_grads(params, bufs, x, y):
    from oracle import numpy_ref as nr
    logits, cache, _ = nr.forward(params, bufs, x, train=True, p=0.0)
    _, dl = nr.cross_entropy(logits, y)
    g = nr.backward(cache, dl)
    # undo the clamp: the DP path defers it until after the all-reduce
    return g


def _clamp_flat(grads, shapes):
    out, o = [], 0
    for k, shp in shapes:
        n = int(np.prod(shp))
        v = grads[o:o + n]
        if k == "spatial.weight":
            v = v.clamp(-1.0, 1.0)
        elif k == "classifier.weight":
            v = v.clamp(-0.25, 0.25)
        out.append(v)
        o += n
    return torch.cat(out)


def _shapes():
    g = Golden("G6")
    return [(k, np.asarray(g.init_params()[k]).shape) for k in PARAM_NAMES]


def _rank_grads(rank, world):
    """Unclamped local gradients of rank's half of the clamp-active G6 batch (CPU oracle as the
    stand-in for the HIP local step; per-rank BN statistics as in DataParallelTrainer)."""
    from oracle import numpy_ref as nr
    g = Golden("G6")
    params, bufs = g.init_params(), g.init_buffers()
    half = g.x.shape[0] // world
    xs, ys = g.x[rank * half:(rank + 1) * half], g.y[rank * half:(rank + 1) * half]
    logits, cache, _ = nr.forward(params, bufs, xs, train=True, p=0.0)
    _, dl = nr.cross_entropy(logits, ys)
    grads = nr.backward(cache, dl * 1000.0)
    dz = dl * 1000.0
    grads["classifier.weight"] = dz.T @ cache["h"]           # undo the oracle's clamp
    ws = params["spatial.weight"].reshape(16, 22).astype(np.float64)
    del ws
    return _flat(grads)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from eegnetreplication_amd import distributed as D
    D.init_process_group("gloo")
    grads = _rank_grads(rank, world)
    D.allreduce_mean_(grads)
    clamped = _clamp_flat(grads, _shapes())
    # fold sharding + gather
    assign = D.lpt_assign([5, 1, 4, 2, 3, 9, 7], world)
    local = {u: rank * 100 + u for u in assign[rank]}
    merged = D.gather_results(local)
    q.put((rank, clamped.numpy(), sorted(merged.items()), assign))
    dist.destroy_process_group()


def test_dp_allreduce_then_clamp_and_fold_sharding():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # every rank ends with the same clamped global-mean gradient
    np.testing.assert_array_equal(res[0][1], res[1][1])
    # and it is clamp(mean(g_r)) -- the clamp sees the global gradient
    g0, g1 = _rank_grads(0, world), _rank_grads(1, world)
    expected = _clamp_flat((g0 + g1) / 2, _shapes())
    np.testing.assert_allclose(res[0][1], expected.numpy(), rtol=1e-12, atol=1e-15)
    cls = slice(sum(int(np.prod(s)) for _, s in _shapes()[:10]), None)
    assert np.max(np.abs(res[0][1][cls][:-4])) <= 0.25 + 1e-12     # classifier.weight (not .bias)
    merged = dict(res[0][2])
    assign = res[0][3]
    assert sorted(merged) == list(range(7))
    for r in range(world):
        for u in assign[r]:
            assert merged[u] == r * 100 + u


def test_lpt_assign_balances_and_is_deterministic():
    from eegnetreplication_amd.distributed import lpt_assign
    costs = [23.0] * 90                     # 90 cross-subject folds, equal cost
    a = lpt_assign(costs, 8)
    assert sorted(sum(a, [])) == list(range(90))
    sizes = sorted(len(x) for x in a)
    assert sizes[-1] - sizes[0] <= 1
    assert a == lpt_assign(costs, 8)
    b = lpt_assign([10, 9, 8, 1, 1, 1], 2)
    loads = [sum([10, 9, 8, 1, 1, 1][i] for i in r) for r in b]
    assert max(loads) - min(loads) <= 4          # optimum for this instance is 13 | 17
