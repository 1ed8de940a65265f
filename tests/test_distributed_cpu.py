"""Multi-process orchestration on CPU (gloo, world_size 2): the product DataParallelTrainer.step
(local step -> ONE all-reduce of [grads | loss | rank 0's BN buffers] -> mean -> clamp -> Adam), and
fold sharding / result gathering.  The device stages are stand-ins here (the local step is the float64 oracle); their HIP
kernels are checked on the GPU in tests/test_gpu_distributed.py."""

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


def _shapes():
    g = Golden("G6")
    return [(k, np.asarray(g.init_params()[k]).shape) for k in PARAM_NAMES]


def _rank_grads(rank, world):
    """Unclamped local gradients of rank's slice of the clamp-active G6 batch (the float64 oracle
    stands in for the HIP local step; per-rank BN statistics as in DataParallelTrainer)."""
    from oracle import numpy_ref as nr
    g = Golden("G6")
    params, bufs = g.init_params(), g.init_buffers()
    half = g.x.shape[0] // world
    xs, ys = g.x[rank * half:(rank + 1) * half], g.y[rank * half:(rank + 1) * half]
    logits, cache, _ = nr.forward(params, bufs, xs, train=True, p=0.0)
    _, dl = nr.cross_entropy(logits, ys)
    return _flat(nr.backward(cache, dl * g.meta["loss_scale"], clamp=False))


def _worker(rank, world, port, q):
    """Drives the product DataParallelTrainer.step (local grads -> reduce -> clamp -> update) on
    CPU/gloo.  Only the device stages are stand-ins: local_grads writes the oracle's unclamped local
    gradient, a rank-specific loss and a rank-specific running-statistics update (what the HIP
    forward does to the BN buffers); clamp / update record what reaches them (the HIP clamp and Adam
    kernels are checked on the GPU: tests/test_gpu_distributed.py)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from eegnetreplication_amd import EEGNet
    from eegnetreplication_amd import distributed as D
    D.init_process_group("gloo")
    torch.manual_seed(100 + rank)                 # different init per rank: the trainer broadcasts
    model = EEGNet(22, 256, p=0.0)
    with torch.no_grad():
        model.flat_bn_buffers().fill_(float(rank + 1))      # rank-specific running statistics
        model.flat_num_batches_tracked().fill_(10 * (rank + 1))
    tr = D.DataParallelTrainer(model)
    calls = []

    def local_grads(x, y, seed, offset):
        calls.append(("local", seed, offset, model.flat_bn_buffers().clone()))
        tr.adam.grads.copy_(_rank_grads(rank, world).float())
        tr.loss.fill_(1.0 + rank)                               # per-rank batch-mean loss
        with torch.no_grad():                                   # the forward's running-stat update
            model.flat_bn_buffers().mul_(0.9).add_(0.1 * (rank + 3))
            model.flat_num_batches_tracked().add_(1)
        return tr.adam.grads

    def clamp(grads):
        calls.append(("clamp", grads.clone()))

    def update(grads):
        calls.append(("update", grads.data_ptr() == tr.adam.grads.data_ptr()))

    tr.local_grads, tr.clamp, tr.update = local_grads, clamp, update
    tr.step(None, None)
    nbt = model.flat_num_batches_tracked().clone()
    # fold sharding + gather
    assign = D.lpt_assign([5, 1, 4, 2, 3, 9, 7], world)
    local = {u: rank * 100 + u for u in assign[rank]}
    merged = D.gather_results(local)
    q.put((rank, [c[0] for c in calls], calls[0][1:3], calls[0][3].numpy(), calls[1][1].numpy(),
           calls[2][1], model.flat_parameters().detach().numpy().copy(), nbt.numpy(),
           sorted(merged.items()), assign, model.flat_bn_buffers().numpy().copy(), float(tr.loss)))
    dist.destroy_process_group()


def test_dp_trainer_step_order_and_fold_sharding():
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
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[1] == ["local", "clamp", "update"]          # clamp after the reduction, then Adam
        assert r[5] is True                                   # Adam consumes the reduced buffer
        np.testing.assert_array_equal(r[3], np.ones_like(r[3]))  # rank 0's BN buffers at construction
        np.testing.assert_array_equal(r[7], [11, 11, 11])        # rank 0's counters, + 1 per step
        # after the step every rank holds rank 0's updated running statistics (DDP broadcast_buffers),
        # carried by the gradient all-reduce (x + 0 == x), and the global-batch mean loss
        np.testing.assert_array_equal(r[10], np.full_like(r[10], np.float32(np.float32(0.9) * 1.0 + np.float32(0.3))))
        assert r[11] == 1.5
    # distinct dropout keys per rank, same seed
    assert res[0][2][0] == res[1][2][0] and res[0][2][1] != res[1][2][1]
    # identical parameters on every rank after the initial broadcast
    np.testing.assert_array_equal(res[0][6], res[1][6])
    # what reaches the clamp is the global-mean gradient (clamp the global gradient)
    g0, g1 = _rank_grads(0, world), _rank_grads(1, world)
    for r in res:
        np.testing.assert_array_equal(r[4], ((g0.float() + g1.float()) * 0.5).numpy())
    merged = dict(res[0][8])
    assign = res[0][9]
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


def _syncbn_worker(rank, world, port, q):
    """DataParallelTrainer(sync_bn=True).step on CPU/gloo with stand-in device stages: stage 2j writes
    a rank-specific fp64 sums vector for pass j, stage 2j + 1 records what the finalize sees."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from eegnetreplication_amd import EEGNet
    from eegnetreplication_amd import distributed as D
    D.init_process_group("gloo")
    torch.manual_seed(7)
    tr = D.DataParallelTrainer(EEGNet(22, 256, p=0.0), sync_bn=True)
    sums = [torch.zeros(n, dtype=torch.float64) for n in (5, 2, 7, 3, 4)]
    tr.stage_sums = lambda B: sums
    seen = []

    def stage(k, x, y, seed, offset, norm_batch):
        j = k // 2
        if k % 2 == 0:
            sums[j].copy_(torch.arange(sums[j].numel(), dtype=torch.float64) * (rank + 1) + 100 * j)
            seen.append(("pass", j, seed, offset, norm_batch))
        else:
            seen.append(("fin", j, sums[j].clone().numpy(), norm_batch))

    tr.stage = stage
    B = 8 - 3 * rank                      # unequal shards (a short last batch on rank 1)
    tr.step(torch.zeros(B, 22, 256), torch.zeros(B, dtype=torch.int64))
    q.put((rank, seen))
    dist.destroy_process_group()


def test_sync_bn_step_reduces_every_pass_before_its_finalize():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_syncbn_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seen in res:
        assert [(e[0], e[1]) for e in seen] == [(s, j) for j in range(5) for s in ("pass", "fin")]
        for e in seen:
            if e[0] == "fin":                     # the finalize sees the sum over ranks of pass j's sums
                j = e[1]
                n = e[2].size
                expect = sum(np.arange(n) * (r + 1) + 100 * j for r in range(world))
                np.testing.assert_array_equal(e[2], expect)
    # one seed, distinct dropout offsets per rank
    p0 = [e for e in res[0][1] if e[0] == "pass"][0]
    p1 = [e for e in res[1][1] if e[0] == "pass"][0]
    assert p0[2] == p1[2] and p0[3] != p1[3]
    # every stage of every rank normalises by the true global batch 8 + 5, not local B x world
    assert {e[-1] for _, seen in res for e in seen} == {13}
