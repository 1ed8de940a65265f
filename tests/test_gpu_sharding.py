"""cfg3 (BASELINE configs[2]: folds sharded over GPUs, no communication) -- the CLI's rank-sharded
path at world 2 (two ranks over gloo on the one GPU; 8-GPU runs are the driver's) against the same
protocol at world 1, and a fold's result against the fold-batch width.

The units are dealt to ranks by ``lpt_assign`` (eegnetreplication_amd/train.py ``_select``), each
rank trains its share as one fold batch (fold-indexed launches) and ``gather_results`` merges them.
Every unit is seeded from its index and a fold-indexed launch splits a fold's batch over workgroups
by the batch size alone, so the merged results must equal the world-1 run bit for bit: test
accuracies, validation accuracies / losses and every tensor of every saved state.  The unit counts
are chosen so that the two runs put different numbers of folds into one launch (18 vs 9, 12 vs 6).

Protocols: within_subject_training (train.py:30-148) and cross_subject_training (train.py:151-291),
on the seeded synthetic sessions (real BCI IV-2a data is absent).
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

EPOCHS = 2


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np_state(sd):
    return {k: v.detach().cpu().numpy().copy() for k, v in sd.items()}


def _run(protocol, max_units):
    import importlib
    T_ = importlib.import_module("eegnetreplication_amd.train")    # (the package exports train())
    if protocol == "ws":
        per_subject, avg, states = T_.within_subject_training(EPOCHS, 0, "cuda:0", 90, max_units)
        return per_subject, avg, [_np_state(s) for s in states], {}
    units = {}
    best, per_subject, avg = T_.cross_subject_training(EPOCHS, 0, "cuda:0", 90, max_units, units_out=units)
    # every fold's record: test / validation accuracy, validation loss and its final state
    per_fold = {u: (r["test_acc"], r["val_acc"], r["val_loss"], _np_state(r["state"])) for u, r in units.items()}
    return per_subject, avg, [_np_state(best)], per_fold


def _worker(rank, world, port, protocol, max_units, data_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", EEGNET_SYNTHETIC="1",
                      EEGNET_DATA_DIR=data_dir)
    import torch.distributed as dist
    from eegnetreplication_amd import distributed as D
    try:
        D.init_process_group("gloo")
        torch.cuda.set_device(0)
        q.put((rank, _run(protocol, max_units), None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:                 # report instead of hanging the parent
        q.put((rank, None, repr(e)))
        raise


def _sharded(protocol, max_units, data_dir, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, protocol, max_units, data_dir, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[2] is None, f"rank {r[0]}: {r[2]}"
    for p in procs:
        assert p.exitcode == 0
    return res


# ("cs", None): BASELINE configs[2] at its own size -- all 90 cross-subject folds, dealt 45 + 45 over
# the two ranks (one launch of 90 folds at world 1 against two of 45)
@pytest.mark.parametrize("protocol,max_units", [("ws", 18), ("cs", 12), ("cs", None)])
def test_sharded_protocol_equals_world1(tmp_path, monkeypatch, protocol, max_units):
    _dev()
    data_dir = str(tmp_path / "nodata")
    monkeypatch.setenv("EEGNET_SYNTHETIC", "1")
    monkeypatch.setenv("EEGNET_DATA_DIR", data_dir)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    one = _run(protocol, max_units)
    res = _sharded(protocol, max_units, data_dir)
    for rank, got, _ in res:                  # gather_results gives every rank the merged results
        assert got[0] == one[0], f"rank {rank}: per-subject test accuracies differ"
        assert got[1] == one[1]
        assert len(got[2]) == len(one[2])
        for sa, sb in zip(got[2], one[2]):
            assert sorted(sa) == sorted(sb)
            for k in sb:
                np.testing.assert_array_equal(sa[k], sb[k], err_msg=f"rank {rank} {protocol}: {k}")
        assert sorted(got[3]) == sorted(one[3])
        if max_units is None and protocol == "cs":
            assert len(one[3]) == 90
        for u, (ta, va, vl, st) in one[3].items():
            tb, vb, wl, sb = got[3][u]
            assert (ta, va, vl) == (tb, vb, wl), f"rank {rank} fold {u}: accuracies / validation loss differ"
            for k in st:
                np.testing.assert_array_equal(sb[k], st[k], err_msg=f"rank {rank} fold {u}: {k}")


def test_fold_result_independent_of_fold_batch_width():
    """The same 12 folds (batch 64, 22 x 257, p = 0.5, a short last batch) trained as one fold batch,
    as three batches of four and one at a time (all fold-indexed launches): identical parameters,
    BN buffers, counters, Adam state and loss sums."""
    from eegnetreplication_amd import EEGNet, FoldBatch
    dev = _dev()
    K, n, Cc, Tt = 12, 150, 22, 257
    rng = np.random.default_rng(8)
    data = [(torch.from_numpy(rng.standard_normal((n, Cc, Tt), dtype=np.float32)).to(dev),
             torch.from_numpy(rng.integers(0, 4, n)).to(dev)) for _ in range(K)]
    seeds = [300 + k for k in range(K)]

    def models():
        torch.manual_seed(21)
        return [EEGNet(Cc, Tt, p=0.5).to(dev) for _ in range(K)]

    def run(widths):
        ms, sums, k0 = models(), [None] * K, 0
        for w in widths:
            ks = list(range(k0, k0 + w))
            fb = FoldBatch([ms[k] for k in ks], [seeds[k] for k in ks], fused=True)
            gens = [torch.Generator().manual_seed(seeds[k]) for k in ks]
            for _ in range(2):
                out = fb.epoch([data[k] for k in ks], 64, gens)
            for k, s in zip(ks, out):
                sums[k] = s
            k0 += w
        torch.cuda.synchronize()
        return [(m.flat_parameters().clone(), m.flat_bn_buffers().clone(),
                 m.flat_num_batches_tracked().clone()) for m in ms], sums

    a, sa = run([12])
    for widths in ([4, 4, 4], [1] * 12):
        b, sb = run(widths)
        for k in range(K):
            assert torch.equal(sa[k], sb[k]), f"widths {widths} fold {k}: loss sums differ"
            for u, v in zip(a[k], b[k]):
                assert torch.equal(u, v), f"widths {widths} fold {k}: state differs"
