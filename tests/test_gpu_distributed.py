"""GPU checks of the data-parallel (cfg4) stages and the standalone kernels they use:
EEGNET_NO_CLAMP, eegnet_clamp_grads (k_clamp), eegnet_adam_step (k_adam + k_step_inc), the CE
inside eegnet_backward, and the product DataParallelTrainer at world_size 1 (against FusedTrainer
and the reference golden vectors) and world_size 2 (two ranks on the one GPU over gloo, against the
float64 oracle's clamp(mean of the per-rank gradients) followed by Adam).

Semantics pinned: clamps of model.py:44 / model.py:84 act on the global gradient, i.e. after the
all-reduce; Adam of train.py:94-101."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

from golden_util import Golden, assert_close, assert_grads_close, assert_params_close
from hip_cases import flat_to_dict

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _model_from(g: Golden, dev):
    from eegnetreplication_amd import EEGNet
    m = g.meta
    model = EEGNet(m["C"], m["T"], F1=m["F1"], D=m["D"], p=m["p"])
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in g.init.items()})
    return model.to(dev).train()


def test_no_clamp_then_clamp_kernel_on_clamp_active_G6():
    """G6 (loss x 1000: spatial grads saturate at +-1, classifier at +-0.25): backward with
    EEGNET_NO_CLAMP returns the raw gradients; eegnet_clamp_grads then gives the reference's
    clamped gradients (golden grad.*)."""
    from eegnetreplication_amd import ops
    from oracle import numpy_ref as nr
    dev = _dev()
    g = Golden("G6")
    model = _model_from(g, dev)
    shape = model.shape
    B = g.x.shape[0]
    x = torch.from_numpy(g.x).to(dev)
    ws = ops.new_workspace(shape, B, dev)
    flat = model.flat_parameters().clone()
    logits = ops.forward_train(shape, flat, model.flat_bn_buffers().clone(), x, ws, 1, 1)
    ref_logits, cache, _ = nr.forward(g.init_params(), g.init_buffers(), g.x, train=True, p=0.0)
    _, dl = nr.cross_entropy(ref_logits, g.y)
    dl = dl * g.meta["loss_scale"]
    raw = ops.backward(shape, flat, x, ws, 1, 1, dlogits=torch.from_numpy(dl.astype(np.float32)).to(dev),
                       clamp=False)
    torch.cuda.synchronize()
    assert_close(logits.cpu().numpy(), g.z["logits"], name="G6 logits")
    ref_raw = nr.backward(cache, dl, clamp=False)
    got_raw = flat_to_dict(model, raw)
    assert np.abs(got_raw["spatial.weight"]).max() > 1.0            # the clamp has work to do
    assert np.abs(got_raw["classifier.weight"]).max() > 0.25
    assert_grads_close(got_raw, ref_raw, prefix="G6 raw grad.")
    ops.clamp_grads(shape, raw)
    torch.cuda.synchronize()
    assert_grads_close(flat_to_dict(model, raw), g.group("grad"), prefix="G6 clamped grad.",
                       unclamped_scale=g.unclamped_scale())


def test_backward_ce_and_standalone_adam_match_golden():
    """eegnet_backward with labels (CE fused into pass C, train.py:103) gives the golden loss and
    grads; eegnet_adam_step on them gives the golden post-Adam parameters and advances the device
    step counter (k_step_inc)."""
    from eegnetreplication_amd import ops
    dev = _dev()
    g = Golden("G1")
    model = _model_from(g, dev)
    shape = model.shape
    B = g.x.shape[0]
    x = torch.from_numpy(g.x).to(dev)
    y = torch.from_numpy(g.y).to(dev)
    ws = ops.new_workspace(shape, B, dev)
    flat = model.flat_parameters()
    ops.forward_train(shape, flat, model.flat_bn_buffers(), x, ws, 1, 1)
    loss = torch.zeros(1, device=dev)
    grads = ops.backward(shape, flat, x, ws, 1, 1, labels=y, loss=loss)
    torch.cuda.synchronize()
    assert abs(float(loss) - float(g.z["loss"])) <= 1e-4 * max(1.0, abs(float(g.z["loss"])))
    assert_grads_close(flat_to_dict(model, grads), g.group("grad"), prefix="G1 grad.")
    n = flat.numel()
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.adam_step(flat, grads, m, v, step, lr=1e-3, betas=(0.9, 0.999), eps=1e-7)
    torch.cuda.synchronize()
    assert int(step.item()) == 1
    assert_params_close({k: p.detach().cpu().numpy() for k, p in model.named_parameters()},
                        g.group("step1"), prefix="G1 step1.")


def test_dp_trainer_world1_matches_fused_and_golden():
    """DataParallelTrainer at world_size 1 (NO_CLAMP local step, k_clamp, k_adam): after one step the
    golden post-Adam parameters; over 3 steps bit-identical to FusedTrainer (whose Adam and clamps
    are fused into the finalizes) -- same parameters, BN buffers, Adam moments and losses."""
    from eegnetreplication_amd import FusedTrainer
    from eegnetreplication_amd.distributed import DataParallelTrainer
    dev = _dev()
    g = Golden("G1")
    x = torch.from_numpy(g.x).to(dev)
    y = torch.from_numpy(g.y).to(dev)
    a, b = _model_from(g, dev), _model_from(g, dev)
    dp, fu = DataParallelTrainer(a), FusedTrainer(b)
    assert dp.world == 1
    for s in range(3):
        la = float(dp.step(x, y))
        lb = float(fu.step(x, y))
        assert la == lb, s
        if s == 0:
            assert_params_close({k: p.detach().cpu().numpy() for k, p in a.named_parameters()},
                                g.group("step1"), prefix="DP step1.")
    torch.cuda.synchronize()
    assert torch.equal(a.flat_parameters(), b.flat_parameters())
    assert torch.equal(a.flat_bn_buffers(), b.flat_bn_buffers())
    assert torch.equal(dp.adam.state, fu.adam.state)
    assert int(dp.adam.step.item()) == int(fu.adam.step.item()) == 3
    assert torch.equal(a.flat_num_batches_tracked(), b.flat_num_batches_tracked())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from eegnetreplication_amd import distributed as D
    try:
        D.init_process_group("gloo")
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        g = Golden("G6")
        model = _model_from(g, dev)
        if rank == 1:                       # the trainer must broadcast rank 0's start point
            with torch.no_grad():
                model.flat_parameters().mul_(0.5)
                model.flat_bn_buffers().add_(1.0)
        tr = D.DataParallelTrainer(model)
        half = g.x.shape[0] // world
        x = torch.from_numpy(g.x[rank * half:(rank + 1) * half]).to(dev)
        y = torch.from_numpy(g.y[rank * half:(rank + 1) * half]).to(dev)
        tr.step(x, y)
        torch.cuda.synchronize()
        q.put((rank, model.flat_parameters().cpu().numpy().copy(), float(tr.loss.item()), None,
               model.flat_bn_buffers().cpu().numpy().copy()))
        dist.destroy_process_group()
    except Exception as e:                 # report instead of hanging the parent
        q.put((rank, None, None, repr(e), None))
        raise


def test_dp_trainer_world2_on_one_gpu():
    """Two ranks (gloo over device tensors, both on cuda:0) run the product DataParallelTrainer on
    the two halves of G6: both end with identical parameters equal to Adam(clamp(mean_r g_r)) of
    the float64 oracle, g_r being rank r's local gradient with its own BN batch statistics."""
    import torch.multiprocessing as mp
    from oracle import numpy_ref as nr
    _dev()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, f"rank {r[0]}: {r[3]}"
    for p in procs:
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][4], res[1][4])      # rank 0's running statistics everywhere
    assert res[0][2] == res[1][2]                             # the global-batch mean loss
    g = Golden("G6")
    params, bufs = g.init_params(), g.init_buffers()
    half = g.x.shape[0] // world
    acc, losses = None, []
    for r in range(world):
        logits, cache, _ = nr.forward(params, bufs, g.x[r * half:(r + 1) * half], train=True, p=0.0)
        lr_, dl = nr.cross_entropy(logits, g.y[r * half:(r + 1) * half])
        losses.append(float(lr_))
        gr = nr.backward(cache, dl, clamp=False)
        acc = gr if acc is None else {k: acc[k] + gr[k] for k in acc}
    mean = {k: v / world for k, v in acc.items()}
    assert abs(res[0][2] - sum(losses) / world) <= 1e-4 * max(1.0, abs(sum(losses) / world))
    mean["spatial.weight"] = np.clip(mean["spatial.weight"], -1.0, 1.0)
    mean["classifier.weight"] = np.clip(mean["classifier.weight"], -0.25, 0.25)
    expect = nr.adam_step(params, mean, nr.adam_init(params))
    from eegnetreplication_amd import EEGNet
    m = EEGNet(g.meta["C"], g.meta["T"])
    got, o = {}, 0
    for k, p in m.named_parameters():
        got[k] = res[0][1][o:o + p.numel()].reshape(p.shape)
        o += p.numel()
    assert_params_close(got, expect, prefix="DP world2 ")


def test_sync_bn_world1_bit_identical_to_fused():
    """DataParallelTrainer(sync_bn=True) at world_size 1: the staged step (each pass with its finalize
    deferred, then k_fin on the sums) is the fused step split at its reductions -- bit-identical
    parameters, BN buffers, counters, Adam state and losses to FusedTrainer over 3 steps."""
    from eegnetreplication_amd import FusedTrainer
    from eegnetreplication_amd.distributed import DataParallelTrainer
    dev = _dev()
    g = Golden("G1")
    x = torch.from_numpy(g.x).to(dev)
    y = torch.from_numpy(g.y).to(dev)
    a, b = _model_from(g, dev), _model_from(g, dev)
    dp, fu = DataParallelTrainer(a, sync_bn=True), FusedTrainer(b)
    for s in range(3):
        la = float(dp.step(x, y))
        lb = float(fu.step(x, y))
        assert la == lb, s
    torch.cuda.synchronize()
    assert torch.equal(a.flat_parameters(), b.flat_parameters())
    assert torch.equal(a.flat_bn_buffers(), b.flat_bn_buffers())
    assert torch.equal(dp.adam.state, fu.adam.state)
    assert torch.equal(a.flat_num_batches_tracked(), b.flat_num_batches_tracked())


def _syncbn_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import torch.distributed as dist
    from eegnetreplication_amd import distributed as D
    try:
        D.init_process_group("gloo")
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        g = Golden("G6")
        model = _model_from(g, dev)
        tr = D.DataParallelTrainer(model, sync_bn=True)
        half = g.x.shape[0] // world
        x = torch.from_numpy(g.x[rank * half:(rank + 1) * half]).to(dev)
        y = torch.from_numpy(g.y[rank * half:(rank + 1) * half]).to(dev)
        losses = [float(tr.step(x, y))]
        torch.cuda.synchronize()
        q.put((rank, model.flat_parameters().cpu().numpy().copy(), losses, None,
               model.flat_bn_buffers().cpu().numpy().copy(), tr.adam.state.cpu().numpy().copy()))
        dist.destroy_process_group()
    except Exception as e:                 # report instead of hanging the parent
        q.put((rank, None, None, repr(e), None, None))
        raise


def test_sync_bn_world2_equals_single_device_on_the_whole_batch():
    """Two ranks (gloo, both on cuda:0) with synchronised BatchNorm on the two halves of G6 take the
    same step as ONE device on the whole batch (FusedTrainer): BN statistics over the global batch,
    global CE mean, clamps on the global gradient, Adam -- running statistics, Adam moments and the
    loss agree to fp32 summation order (rtol 1e-5), the parameters within assert_params_close (gamma1 /
    beta1 take an O(lr) Adam step on rounding residue), and both ranks are identical."""
    import torch.multiprocessing as mp
    from eegnetreplication_amd import FusedTrainer
    dev = _dev()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_syncbn_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, f"rank {r[0]}: {r[3]}"
    for p in procs:
        assert p.exitcode == 0
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][4], res[1][4])
    np.testing.assert_array_equal(res[0][5], res[1][5])
    assert res[0][2] == res[1][2]
    g = Golden("G6")
    m = _model_from(g, dev)
    fu = FusedTrainer(m)
    x, y = torch.from_numpy(g.x).to(dev), torch.from_numpy(g.y).to(dev)
    ref_losses = [float(fu.step(x, y))]
    torch.cuda.synchronize()
    np.testing.assert_allclose(res[0][2], ref_losses, rtol=1e-5)
    assert_params_close(flat_to_dict(m, torch.from_numpy(res[0][1])), flat_to_dict(m, m.flat_parameters()),
                        prefix="SyncBN world2 ")
    for got, ref, what in ((res[0][4], m.flat_bn_buffers(), "bn"), (res[0][5], fu.adam.state, "adam")):
        ref = ref.detach().cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * float(np.abs(ref).max()), err_msg=what)


def _rccl_worker(port, q):
    """World 1 over the nccl (= RCCL) backend in a fresh process: DataParallelTrainer runs its real
    collectives (broadcast of the start point, the per-step all-reduce of [grads | loss | buffers],
    the sync-BN batch and per-pass sums) through RCCL on the device."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from eegnetreplication_amd import FusedTrainer
    from eegnetreplication_amd.distributed import DataParallelTrainer
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        out = {"backend": str(dist.get_backend())}
        g = Golden("G1")
        x = torch.from_numpy(g.x).to(dev)
        y = torch.from_numpy(g.y).to(dev)
        for sync in (False, True):
            a, b = _model_from(g, dev), _model_from(g, dev)
            dp, fu = DataParallelTrainer(a, sync_bn=sync), FusedTrainer(b)
            same_loss = all(float(dp.step(x, y)) == float(fu.step(x, y)) for _ in range(3))
            torch.cuda.synchronize()
            out[sync] = (dp.dist, same_loss, torch.equal(a.flat_parameters(), b.flat_parameters()),
                         torch.equal(a.flat_bn_buffers(), b.flat_bn_buffers()),
                         torch.equal(dp.adam.state, fu.adam.state))
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:                 # report instead of hanging the parent
        q.put((None, repr(e)))
        raise


def test_dp_trainer_over_rccl_world1():
    """The RCCL (backend "nccl") branch on the one-GPU box: at world 1 every collective is an identity,
    so DataParallelTrainer -- plain and sync_bn -- stays bit-identical to FusedTrainer over 3 steps
    while each of its broadcasts and all-reduces runs through RCCL."""
    import torch.multiprocessing as mp
    _dev()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    out, err = q.get(timeout=150)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    for sync in (False, True):
        assert out[sync] == (True, True, True, True, True), (sync, out[sync])
