"""Fold-batched training (eegnetreplication_amd.folds.FoldBatch) on the GPU.

FoldBatch only interleaves independent steps (per-fold HIP streams running FusedTrainer's step, or
fold-indexed launches), so the bar is bit-equality: every fold of a concurrent batch must end with
exactly the parameters, BN buffers, Adam state and loss sums of the same fold trained alone, and a
one-fold stream batch must reproduce FusedTrainer, whose step is pinned to the oracle and the
reference golden vectors by tests/test_gpu_parity.py.  A fold-indexed launch splits a fold's batch
over fewer workgroups than FusedTrainer (by the batch size alone: eegnet_host.hip fold_tpw), so
against FusedTrainer it agrees to the fp32 rounding of its partial sums, not bit for bit.
Shapes follow the real protocol: 22 x 257 trials (02_preprocessing_pipeline.ipynb:1867), batch 64
with a short last batch (train.py:87, DataLoader drop_last=False).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

C, T = 22, 257
PARAMS = ("temporal.0.weight", "temporal.1.weight", "temporal.1.bias", "spatial.weight",
          "aggregation.0.weight", "aggregation.0.bias", "block_2.0.weight", "block_2.1.weight",
          "block_2.2.weight", "block_2.2.bias", "classifier.weight", "classifier.bias")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _data(n, seed, dev):
    rng = np.random.default_rng(seed)
    X = torch.from_numpy(rng.standard_normal((n, C, T), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.integers(0, 4, n).astype(np.int64)).to(dev)
    return X, y


def _models(k, p, dev):
    from eegnetreplication_amd import EEGNet
    torch.manual_seed(7)
    out = []
    for _ in range(k):
        out.append(EEGNet(C, T, p=p).to(dev))
    return out


def _clone(m, p, dev):
    from eegnetreplication_amd import EEGNet
    c = EEGNet(C, T, p=p)
    c.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    return c.to(dev)


def _state(fb, k):
    m = fb.models[k]
    return (m.flat_parameters().clone(), m.flat_bn_buffers().clone(), fb.adam[k].state.clone(),
            m.flat_num_batches_tracked().clone())


def test_concurrent_folds_equal_each_fold_alone():
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    sizes, seeds = [200, 130, 69], [11, 22, 33]
    data = [_data(n, 100 + i, dev) for i, n in enumerate(sizes)]
    models = _models(3, 0.5, dev)
    alone = [_clone(m, 0.5, dev) for m in models]
    fb = FoldBatch(models, seeds)
    gens = [torch.Generator().manual_seed(s) for s in seeds]
    sums_all = [fb.epoch(data, 64, gens) for _ in range(2)]
    torch.cuda.synchronize()
    for k in range(3):
        one = FoldBatch([alone[k]], [seeds[k]], fused=False)      # the same per-fold stream path
        g = [torch.Generator().manual_seed(seeds[k])]
        sums_one = [one.epoch([data[k]], 64, g) for _ in range(2)]
        torch.cuda.synchronize()
        for a, b in zip(_state(fb, k), _state(one, 0)):
            assert torch.equal(a, b), f"fold {k}: concurrent run differs from the fold alone"
        for e in range(2):
            assert torch.equal(sums_all[e][k], sums_one[e][0]), f"fold {k} epoch {e}: loss sums differ"
        assert np.isfinite(float(sums_one[1][0]))
        assert int(fb.adam[k].step.item()) == 2 * ((sizes[k] + 63) // 64)


@pytest.mark.parametrize("fused", [False, True])
def test_single_fold_matches_fused_trainer(fused):
    """fused=False (one stream per fold): FusedTrainer's launches, bit for bit.  fused=True (a
    fold-indexed launch, fewer workgroups per fold): the same step to fp32 rounding -- parameters
    at golden_util's post-Adam tolerance, the BN1 / BN3 running statistics at rtol 1e-4 (BN2's
    follow gamma1 / beta1, whose gradients are rounding residue: DESIGN 7)."""
    from golden_util import assert_params_close
    from eegnetreplication_amd import FoldBatch, FusedTrainer
    dev = _dev()
    X, y = _data(150, 5, dev)
    (m,) = _models(1, 0.0, dev)           # p = 0: the dropout key stream does not matter
    ref = _clone(m, 0.0, dev)
    fb = FoldBatch([m], [1], fused=fused)
    fb.epoch([(X, y)], 64, [torch.Generator().manual_seed(3)])
    from eegnetreplication_amd.dataset import epoch_permutation
    perm = epoch_permutation(150, torch.Generator().manual_seed(3)).to(dev)
    tr = FusedTrainer(ref)
    for i in range(0, 150, 64):
        idx = perm[i:i + 64]
        tr.step(X.index_select(0, idx), y.index_select(0, idx))
    torch.cuda.synchronize()
    if not fused:
        assert torch.equal(m.flat_parameters(), ref.flat_parameters())
        assert torch.equal(m.flat_bn_buffers(), ref.flat_bn_buffers())
        assert torch.equal(fb.adam[0].state, tr.adam.state)
        return
    assert_params_close({k: p.detach().cpu().numpy() for k, p in m.named_parameters()},
                        {k: p.detach().cpu().numpy() for k, p in ref.named_parameters()}, steps=3,
                        rtol=1e-4, atol_frac=1e-4, prefix="fold launch vs FusedTrainer ")
    from golden_util import assert_close
    bm, br = dict(m.named_buffers()), dict(ref.named_buffers())
    for k in ("temporal.1.running_mean", "temporal.1.running_var", "block_2.2.running_mean",
              "block_2.2.running_var"):
        assert_close(bm[k].cpu().numpy(), br[k].cpu().numpy(), atol_frac=1e-4, name=k)
    assert torch.equal(m.flat_num_batches_tracked(), ref.flat_num_batches_tracked())


def test_graph_replay_equals_eager():
    """graphs=True: epoch 1 eager + capture, later epochs replay the captured graph.  Dropout keys
    follow the device step, so replays must match an all-eager run bit for bit."""
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    sizes, seeds = [150, 100], [5, 6]
    data = [_data(n, 200 + i, dev) for i, n in enumerate(sizes)]
    models = _models(2, 0.5, dev)
    twins = [_clone(m, 0.5, dev) for m in models]
    eager = FoldBatch(models, seeds)
    graph = FoldBatch(twins, seeds, graphs=True)
    ge = [torch.Generator().manual_seed(s) for s in seeds]
    gg = [torch.Generator().manual_seed(s) for s in seeds]
    for e in range(3):
        se = eager.epoch(data, 64, ge)
        sg = graph.epoch(data, 64, gg)
        torch.cuda.synchronize()
        for k in range(2):
            assert torch.equal(se[k], sg[k]), f"epoch {e} fold {k}: loss sums differ"
            for a, b in zip(_state(eager, k), _state(graph, k)):
                assert torch.equal(a, b), f"epoch {e} fold {k}: graph replay differs from eager"
    assert all(graph._graph[k] is not None for k in range(2))
    assert int(graph.adam[0].step.item()) == 3 * 3


def test_step_keyed_dropout_changes_every_step():
    """With keys from the device step, a replayed step must not reuse the previous step's masks:
    two steps on the same batch from the same weights differ only through the step counter."""
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    X, y = _data(64, 9, dev)
    (m,) = _models(1, 0.5, dev)
    a, b = _clone(m, 0.5, dev), _clone(m, 0.5, dev)
    fa, fb = FoldBatch([a], [1]), FoldBatch([b], [1])
    fb.adam[0].step.fill_(1)               # same weights and moments, next step's key
    la = fa.epoch([(X, y)], 64)[0]
    lb = fb.epoch([(X, y)], 64)[0]
    torch.cuda.synchronize()
    assert not torch.equal(la, lb), "dropout masks did not change with the step counter"


def test_protocol_fold_batch_matches_one_at_a_time():
    """train.py's protocol runner: _run_folds (FoldBatch, fold-indexed launches, graphs) against
    _run_fold (the reference-shaped train() + evaluate_model() loop, model.py:101-227) on the same
    units.  With p = 0 the dropout keying is moot; the two split each batch over different
    workgroup counts, so weights agree to fp32 rounding and accuracies to one trial; a second
    fold-batched run reproduces the first bit for bit."""
    import importlib
    T_ = importlib.import_module("eegnetreplication_amd.train")   # (the package exports train())
    dev = _dev()
    rng = np.random.default_rng(4)
    specs = []
    for u in range(3):
        X = rng.standard_normal((150, C, T)).astype(np.float64)
        y = rng.integers(0, 4, 150).astype(np.int64)
        ids = rng.permutation(150)
        te = (rng.standard_normal((40, C, T)), rng.integers(0, 4, 40).astype(np.int64))
        specs.append((X, y, ids[:100], ids[100:], te, 0.0, 10 + u))
    from golden_util import assert_params_close
    batched = T_._run_units(specs, 3, dev, fold_batch=3)
    single = T_._run_units(specs, 3, dev, fold_batch=0)
    for k, (a, b) in enumerate(zip(batched, single)):
        # one trial of 40 / 50 may flip on fp32 rounding of the fold launch's partial sums
        assert abs(a["test_acc"] - b["test_acc"]) <= 100 / 40 + 1e-9, k
        assert abs(a["val_acc"] - b["val_acc"]) <= 100 / 50 + 1e-9, k
        assert abs(a["val_loss"] - b["val_loss"]) <= 1e-4 * abs(b["val_loss"]), k
        assert_params_close({n: a["state"][n].numpy() for n in PARAMS},
                            {n: b["state"][n].numpy() for n in PARAMS}, steps=6, rtol=1e-4,
                            atol_frac=1e-4, prefix=f"unit {k} ")
    again = T_._run_units(specs, 3, dev, fold_batch=3)    # fold batches are bit-reproducible
    for a, b in zip(batched, again):
        assert a["test_acc"] == b["test_acc"] and a["val_loss"] == b["val_loss"]
        for n in b["state"]:
            assert torch.equal(a["state"][n], b["state"][n])


@pytest.mark.parametrize("sizes", [[64, 30, 128], [1, 65]])
def test_graph_fold_edge_sizes(sizes):
    """Edge fold sizes: exactly one batch, a fold smaller than one batch, an exact multiple of 64,
    a single trial, and 64 + 1 (a one-trial last batch).  Graph replays must match eager runs."""
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    seeds = [70 + i for i in range(len(sizes))]
    data = [_data(n, 300 + i, dev) for i, n in enumerate(sizes)]
    models = _models(len(sizes), 0.5, dev)
    twins = [_clone(m, 0.5, dev) for m in models]
    eager, graph = FoldBatch(models, seeds), FoldBatch(twins, seeds, graphs=True)
    ge = [torch.Generator().manual_seed(s) for s in seeds]
    gg = [torch.Generator().manual_seed(s) for s in seeds]
    for _ in range(2):
        se, sg = eager.epoch(data, 64, ge), graph.epoch(data, 64, gg)
        torch.cuda.synchronize()
        for k in range(len(sizes)):
            assert torch.equal(se[k], sg[k])
            for a, b in zip(_state(eager, k), _state(graph, k)):
                assert torch.equal(a, b)
            assert np.isfinite(float(sg[k]))


@pytest.mark.parametrize("graphs", [False, True])
def test_fused_fold_launch_equals_per_fold_streams(graphs):
    """eegnet_train_step_folds (all folds in one launch per pass, fold = grid y) against the same
    folds each in a one-fold fold-indexed launch: identical parameters, BN buffers, counters, Adam
    state and loss sums, epoch after epoch (equal-size folds, a short last batch, p = 0.5)."""
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    K, n = 5, 150
    seeds = [40 + k for k in range(K)]
    data = [_data(n, 500 + k, dev) for k in range(K)]
    models = _models(K, 0.5, dev)
    twins = [_clone(m, 0.5, dev) for m in models]
    fused = FoldBatch(models, seeds, graphs=graphs, fused=True)
    alone = [FoldBatch([t], [s], graphs=graphs, fused=True) for t, s in zip(twins, seeds)]
    gf = [torch.Generator().manual_seed(s) for s in seeds]
    gs = [torch.Generator().manual_seed(s) for s in seeds]
    for e in range(3):
        sf = fused.epoch(data, 64, gf)
        ss = [fb.epoch([data[k]], 64, [gs[k]])[0] for k, fb in enumerate(alone)]
        torch.cuda.synchronize()
        for k in range(K):
            assert torch.equal(sf[k], ss[k]), f"epoch {e} fold {k}: loss sums differ"
            for a, b in zip(_state(fused, k), _state(alone[k], 0)):
                assert torch.equal(a, b), f"epoch {e} fold {k}: 5-fold launch differs from the fold alone"
    assert fused._fz is not None and (fused._fz["graph"] is not None) == graphs
    assert int(fused.adam[0].step.item()) == 3 * 3


@pytest.mark.parametrize("B", [64, 1440])
def test_padded_x_rows_bit_identical(B):
    """x rows at pitch 260 (ops.pad_x_rows; the 22 x 257 kernels then DMA them in 16-byte units plus
    one trailing dword instead of five dword pieces) train bit-identically to contiguous x: same
    parameters, BN buffers, Adam state and losses over three fused steps."""
    from eegnetreplication_amd import FusedTrainer, ops
    dev = _dev()
    X, y = _data(B, 11, dev)
    assert _models(1, 0.5, dev)[0].shape.x_pitch() == 260
    Xp = ops.pad_x_rows(X, 260)
    assert ops.x_pitch_of(Xp) == 260 and torch.equal(Xp, X)
    outs = []
    for xin in (X, Xp):
        m = _models(1, 0.5, dev)[0]
        tr = FusedTrainer(m)
        losses = [tr.step(xin, y).clone() for _ in range(3)]
        torch.cuda.synchronize()
        outs.append((m.flat_parameters().clone(), m.flat_bn_buffers().clone(), tr.adam.state.clone(),
                     torch.cat(losses)))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_in_place_x_update_is_seen_by_the_padded_fold_launch():
    """22 x 257 fold launches train from a padded copy of each fold's X (FoldBatch._fused_state).  A
    caller that refills X in place between epochs (a preallocated augmentation buffer) must train on
    the new values: graphed fold launches over an X mutated in place equal, bit for bit, the same
    folds trained on a fresh tensor holding the new values."""
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    X0, y = _data(192, 31, dev)
    X1, _ = _data(192, 32, dev)
    runs = []
    for mode in ("in_place", "fresh"):
        models = _models(2, 0.5, dev)
        fb = FoldBatch(models, [5, 6], graphs=True, fused=True)
        gens = [torch.Generator().manual_seed(s) for s in (5, 6)]
        X = X0.clone()
        fb.epoch([(X, y)] * 2, 64, gens)             # eager epoch on X0 (pads, captures)
        if mode == "in_place":
            X.copy_(X1)                              # same tensor, new values
            Xe = X
        else:
            Xe = X1.clone()                          # a new tensor: new state, new padded copy
        fb.epoch([(Xe, y)] * 2, 64, gens)
        fb.epoch([(Xe, y)] * 2, 64, gens)
        torch.cuda.synchronize()
        runs.append([_state(fb, k) for k in range(2)])
    for k in range(2):
        for a, b in zip(runs[0][k], runs[1][k]):
            assert torch.equal(a, b), f"fold {k}: the in-place update of X was not seen"


def _x_stats_numpy(x, K1=32):
    """float64 restatement of eegnet_x_stats for trials x [N, C, T]: [G0 K1][S0][H][Tl][hs R][ts P]
    (G0[d] = sum_c sum_{t<T} X[t] X[t+d] with X[t] = x[t - P] zero outside [0, T))."""
    N, Cc, Tt = x.shape
    P, R = (K1 - 1) // 2, K1 - 1 - (K1 - 1) // 2
    xp = np.zeros((N, Cc, Tt + P + K1), dtype=np.float64)
    xp[:, :, P:P + Tt] = x
    G0 = np.stack([(xp[:, :, :Tt] * xp[:, :, d:d + Tt]).sum(axis=(1, 2)) for d in range(K1)], axis=1)
    S0 = xp[:, :, :Tt].sum(axis=(1, 2))[:, None]
    H = [(x[:, :, a] * x[:, :, b]).sum(axis=1) for a in range(R) for b in range(a, R)]
    Tl = [(x[:, :, Tt - P + u] * x[:, :, Tt - P + v]).sum(axis=1) for u in range(P) for v in range(u, P)]
    hs = [x[:, :, a].sum(axis=1) for a in range(R)]
    ts = [x[:, :, Tt - P + u].sum(axis=1) for u in range(P)]
    return np.concatenate([G0, S0, np.stack(H + Tl + hs + ts, axis=1)], axis=1)


@pytest.mark.parametrize("Tt,pitched", [(256, False), (257, False), (257, True)])
def test_x_stats_match_numpy(Tt, pitched):
    """eegnet_x_stats (per-trial BN1 lag sums, window sums, edge products) against a float64 numpy
    restatement, for the recordings' 22 x 257 (contiguous and at the 260-float pitch) and 22 x 256."""
    from eegnetreplication_amd import EEGNet, ops
    dev = _dev()
    rng = np.random.default_rng(19)
    x = rng.standard_normal((37, C, Tt)).astype(np.float32)
    X = torch.from_numpy(x).to(dev)
    shape = EEGNet(C, Tt).shape
    if pitched:
        X = ops.pad_x_rows(X, shape.x_pitch())
    got = ops.x_stats(shape, X).cpu().numpy()
    ref = _x_stats_numpy(x.astype(np.float64))
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


def test_fold_launch_with_x_stats_matches_recomputed():
    """Fold launches reading the per-trial BN1 table (FoldBatch(xstats=True), the default) against
    the same folds recomputing the lag-Gram from x every step (xstats=False): the same training to
    fp32 rounding (the batch sums are formed in another order), over three epochs at p = 0; and the
    table follows an in-place change of X."""
    from golden_util import assert_params_close
    from eegnetreplication_amd import FoldBatch
    dev = _dev()
    data = [_data(150, 700 + k, dev) for k in range(3)]
    runs = []
    for xs in (True, False):
        models = _models(3, 0.0, dev)
        fb = FoldBatch(models, [1, 2, 3], graphs=True, fused=True, xstats=xs)
        gens = [torch.Generator().manual_seed(s) for s in (1, 2, 3)]
        Xs = [(X.clone(), y) for X, y in data]
        for e in range(3):
            if e == 2:
                Xs[1][0].mul_(0.5)                   # in place: the table must be recomputed
            fb.epoch(Xs, 64, gens)
        torch.cuda.synchronize()
        runs.append(fb)
    for k in range(3):
        a, b = runs[0].models[k], runs[1].models[k]
        assert_params_close({n: p.detach().cpu().numpy() for n, p in a.named_parameters()},
                            {n: p.detach().cpu().numpy() for n, p in b.named_parameters()}, steps=9,
                            rtol=1e-4, atol_frac=1e-4, prefix=f"fold {k} xstats vs recomputed ")


@pytest.mark.parametrize("T_", [256, 257])
def test_untracked_x_write_needs_invalidate(T_):
    """A write to X through ``X.data`` does not bump X._version, so FoldBatch cannot see it; after
    ``invalidate_x()`` the graphed fold launches (per-trial BN1 table, and at 22 x 257 the padded
    copy) train on the new values -- bit for bit what a fresh FoldBatch on them trains."""
    from eegnetreplication_amd import EEGNet, FoldBatch
    dev = _dev()
    rng = np.random.default_rng(41)
    X0 = torch.from_numpy(rng.standard_normal((128, C, T_), dtype=np.float32)).to(dev)
    X1 = torch.from_numpy(rng.standard_normal((128, C, T_), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.integers(0, 4, 128)).to(dev)
    runs = []
    for mode in ("data_write", "fresh"):
        torch.manual_seed(9)
        models = [EEGNet(C, T_, p=0.0).to(dev).train() for _ in range(2)]
        fb = FoldBatch(models, [3, 4], graphs=True, fused=True, xstats=True)
        gens = [torch.Generator().manual_seed(s) for s in (3, 4)]
        X = X0.clone()
        fb.epoch([(X, y)] * 2, 64, gens)
        if mode == "data_write":
            ver = X._version
            X.data.copy_(X1)                         # not seen by the version counter
            assert X._version == ver
            fb.invalidate_x()
            Xe = X
        else:
            Xe = X1.clone()
        fb.epoch([(Xe, y)] * 2, 64, gens)
        fb.epoch([(Xe, y)] * 2, 64, gens)
        torch.cuda.synchronize()
        runs.append([_state(fb, k) for k in range(2)])
    for k in range(2):
        for a, b in zip(runs[0][k], runs[1][k]):
            assert torch.equal(a, b), f"fold {k}: the X.data write was not picked up after invalidate_x()"
