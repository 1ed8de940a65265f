"""CPU checks of the training-protocol host logic (no GPU): the fold splits the reference's
train.py produces (pinned by values computed in the survey container with the pinned sklearn /
numpy RandomState), the synthetic data feed and the report schema."""

from __future__ import annotations

import hashlib
import json

import numpy as np


def test_within_subject_kfold_split_sizes_and_first_test_ids():
    from sklearn.model_selection import KFold
    X = np.zeros((576, 1))
    splits = list(KFold(n_splits=4, shuffle=True, random_state=42).split(X))
    tv, te = splits[0]
    nval = len(tv) // 5
    assert (len(tv) - nval, nval, len(te)) == (346, 86, 144)
    assert list(te[:5]) == [0, 2, 6, 9, 10]


def test_cross_subject_fold_permutations():
    from eegnetreplication_amd.train import cross_subject_units
    units = cross_subject_units()
    assert len(units) == 90
    assert units[0][2] == [5, 9, 7, 8, 4] and units[0][3] == [3, 2, 6]
    assert units[-1][2] == [1, 6, 4, 5, 7] and units[-1][3] == [8, 3, 2]
    for s, k, tr, va in units:
        assert s not in tr + va and len(set(tr + va)) == 8
    # all 90 folds, pinned by the survey's digest of [subject, repeat (0-based), train, val]
    # rows serialised with json.dumps (sha256 f35bda7822d73141...)
    rows = [[s, (k - 1) % 10, tr, va] for s, k, tr, va in units]
    digest = hashlib.sha256(json.dumps(rows).encode()).hexdigest()
    assert digest.startswith("f35bda7822d73141"), digest


def test_missing_data_raises_unless_synthetic(tmp_path, monkeypatch):
    """dataset.py:266-267: no preprocessed file -> ValueError.  Synthetic sessions are opt-in."""
    import pytest
    from eegnetreplication_amd import dataset as ds
    monkeypatch.setenv("EEGNET_DATA_DIR", str(tmp_path))
    monkeypatch.delenv("EEGNET_SYNTHETIC", raising=False)
    with pytest.raises(ValueError, match="No preprocessed files"):
        ds.build_dataset_from_preprocessed(subject=1)
    with pytest.raises(ValueError, match="Unknown source"):
        ds.build_dataset_from_preprocessed("zenodo", subject=1)
    monkeypatch.setenv("EEGNET_SYNTHETIC", "1")
    assert ds.build_dataset_from_preprocessed(subject=1).X.shape == (288, 22, 257)
    # real files win over the synthetic generator; positional src as in the reference
    X = np.random.default_rng(0).standard_normal((5, 22, 257))
    np.savez(tmp_path / "A02E.npz", X=X, y=np.arange(5) % 4)
    d = ds.build_dataset_from_preprocessed("kaggle", 2, "Eval")
    assert np.array_equal(d.X, X) and d.y.tolist() == [0, 1, 2, 3, 0]
    allv = ds.build_dataset_from_preprocessed(subject="all", mode="Eval")
    assert allv.X.shape[0] == 8 * 288 + 5


def test_synthetic_sessions_shape_and_determinism():
    from eegnetreplication_amd.dataset import build_dataset_from_preprocessed
    a = build_dataset_from_preprocessed(subject=3, synthetic=True)
    b = build_dataset_from_preprocessed(subject=3, synthetic=True)
    e = build_dataset_from_preprocessed(subject=3, mode="Eval", synthetic=True)
    assert a.X.shape == (288, 22, 257) and a.X.dtype == np.float64
    assert np.array_equal(a.X, b.X) and np.array_equal(a.y, b.y)
    assert not np.array_equal(a.X, e.X)
    assert sorted(set(a.y.tolist())) == [0, 1, 2, 3]
    x, y = a[5]
    assert x.shape == (22, 257) and isinstance(y, int)


def test_report_schema(tmp_path):
    from eegnetreplication_amd.train import generate_cs_report, generate_ws_report
    acc = [60.0, 55.5, 70.25, 40.0, 45.0, 50.0, 65.0, 66.0, 72.0]
    p = generate_ws_report(acc, float(np.mean(acc)), [None] * 9, str(tmp_path))
    r = json.load(open(p))
    assert r["training_type"] == "Within-Subject"
    assert set(r) == {"training_type", "timestamp", "model_parameters", "overall_results",
                      "per_subject_results", "model_info", "summary_statistics"}
    assert r["per_subject_results"][0] == {"subject_id": 1, "test_accuracy": 60.0,
                                           "model_saved": "subject_01_best_model.pth",
                                           "performance_rank": 5}
    p = generate_cs_report(None, acc, float(np.mean(acc)), str(tmp_path))
    r = json.load(open(p))
    assert r["model_parameters"]["total_folds"] == 90
    assert r["per_subject_results"][8]["performance_rank"] == 1
    assert (tmp_path / "latest_cross_subject_report.json").exists()


def test_fold_batch_dispatch_chunks_units(monkeypatch):
    """train._run_units: fold_batch <= 1 runs units one by one through _run_fold (the
    reference-shaped train()/evaluate_model() loop); fold_batch = k hands chunks of k units, in
    order, to _run_folds (FoldBatch).  Results come back in unit order either way."""
    import importlib
    T_ = importlib.import_module("eegnetreplication_amd.train")
    calls = []
    monkeypatch.setattr(T_, "_run_fold", lambda *a: calls.append(("one", a[7])) or {"seed": a[7]})
    monkeypatch.setattr(T_, "_run_folds",
                        lambda specs, e, d: calls.append(("batch", [s[6] for s in specs]))
                        or [{"seed": s[6]} for s in specs])
    specs = [(None, None, None, None, None, 0.5, 100 + i) for i in range(7)]
    out = T_._run_units(specs, 3, "cuda", 0)
    assert [r["seed"] for r in out] == list(range(100, 107))
    assert calls == [("one", 100 + i) for i in range(7)]
    calls.clear()
    out = T_._run_units(specs, 3, "cuda", 3)
    assert [r["seed"] for r in out] == list(range(100, 107))
    assert calls == [("batch", [100, 101, 102]), ("batch", [103, 104, 105]), ("batch", [106])]


def test_device_loader_matches_dataloader_shuffle():
    """DeviceLoader(shuffle=True, generator=g) yields the batches DataLoader(batch_size=64,
    shuffle=True, generator=g) yields (train.py:87-89: RandomSampler draws torch.randperm(n, g) per
    epoch; default collate, drop_last=False) -- same trials, same order, over several epochs.
    FoldBatch.epoch draws its permutation the same way (torch.randperm(n, generator=g))."""
    import torch
    from torch.utils.data import DataLoader
    from eegnetreplication_amd.dataset import BCICI2ADataset, DeviceLoader
    rng = np.random.default_rng(5)
    X = rng.standard_normal((150, 3, 8))
    y = rng.integers(0, 4, 150)
    ref = DataLoader(BCICI2ADataset(X, y), batch_size=64, shuffle=True,
                     generator=torch.Generator().manual_seed(7))
    mine = DeviceLoader(X, y, 64, shuffle=True, device="cpu", generator=torch.Generator().manual_seed(7))
    assert len(mine) == len(ref) == 3
    for _ in range(3):
        got = list(mine)
        exp = list(ref)
        assert [len(b[1]) for b in got] == [64, 64, 22]
        for (xa, ya), (xb, yb) in zip(got, exp):
            assert torch.equal(ya, yb)
            assert torch.equal(xa, xb.float())
    # unshuffled loaders (validation / test, train.py:88-89) keep the dataset order
    plain = DataLoader(BCICI2ADataset(X, y), batch_size=64, shuffle=False)
    for (xa, ya), (xb, yb) in zip(DeviceLoader(X, y, 64, device="cpu"), plain):
        assert torch.equal(ya, yb) and torch.equal(xa, xb.float())


def test_fold_batches_are_balanced(monkeypatch):
    """_run_units splits the units into balanced fold batches of at most fold_batch (90 at 48: 45 + 45, not 48 + 42),
    in unit order, and returns the results in unit order."""
    import importlib
    T_ = importlib.import_module("eegnetreplication_amd.train")   # (the package exports train())
    seen = []

    def fake_run_folds(specs, epochs, device):
        seen.append(len(specs))
        return [sp for sp in specs]

    monkeypatch.setattr(T_, "_run_folds", fake_run_folds)
    specs = list(range(90))
    assert T_._run_units(specs, 1, "cpu", 48) == specs
    assert seen == [45, 45]
    seen.clear()
    assert T_._run_units(list(range(36)), 1, "cpu", 48) == list(range(36))
    assert seen == [36]
    seen.clear()
    assert T_._run_units(list(range(10)), 1, "cpu", 4) == list(range(10))
    assert seen == [4, 4, 2]


def _fake_unit(spec):
    """A stand-in unit result that depends only on the unit's spec (as a seeded fold does)."""
    X, y, tr_ids, va_ids, te, p, seed = spec
    return {"test_acc": float(seed) + 0.5, "val_acc": float(len(tr_ids)), "val_loss": p,
            "state": {"w": np.full(3, seed)}}


def test_failed_unit_is_retried_from_a_fresh_state(monkeypatch):
    """a fold is an idempotent unit and is re-run on a host-side failure.  One unit fails
    once (one at a time), and one fold batch fails once (fold-batched); both runs complete with the
    results of a run without failures.  A device fault is not retried."""
    import pytest
    import importlib
    T_ = importlib.import_module("eegnetreplication_amd.train")
    specs = [(None, None, list(range(10 + u)), [], None, 0.5, 100 + u) for u in range(5)]
    ref = [_fake_unit(sp) for sp in specs]
    calls = {"n": 0}

    def flaky_fold(X, y, tr_ids, va_ids, te, p, epochs, seed, device):
        calls["n"] += 1
        if seed == 102 and calls.setdefault("failed", 0) == 0:
            calls["failed"] = 1
            raise RuntimeError("injected host-side failure")
        return _fake_unit((X, y, tr_ids, va_ids, te, p, seed))

    monkeypatch.setattr(T_, "_run_fold", flaky_fold)
    got = T_._run_units(specs, 1, "cpu", fold_batch=0)
    assert calls["failed"] == 1 and calls["n"] == 6
    assert [r["test_acc"] for r in got] == [r["test_acc"] for r in ref]

    state = {"failed": 0, "batches": []}

    def flaky_folds(batch, epochs, device):
        state["batches"].append([sp[6] for sp in batch])
        if state["failed"] == 0 and any(sp[6] == 103 for sp in batch):
            state["failed"] = 1
            raise ValueError("injected failure inside a fold batch")
        return [_fake_unit(sp) for sp in batch]

    monkeypatch.setattr(T_, "_run_folds", flaky_folds)
    got = T_._run_units(specs, 1, "cpu", fold_batch=3)
    assert state["batches"] == [[100, 101, 102], [103, 104], [103, 104]]
    assert [r["test_acc"] for r in got] == [r["test_acc"] for r in ref]

    def gpu_fault(batch, epochs, device):
        raise RuntimeError("HIP error: an illegal memory access was encountered")

    monkeypatch.setattr(T_, "_run_folds", gpu_fault)
    with pytest.raises(RuntimeError, match="HIP error"):
        T_._run_units(specs, 1, "cpu", fold_batch=3)


def test_retry_only_host_failures_on_a_usable_device(monkeypatch):
    """A programming error (TypeError) is not retried, and neither is any failure after which the
    device is unusable (a stream left in graph capture, a failing synchronise)."""
    import pytest
    import importlib
    T_ = importlib.import_module("eegnetreplication_amd.train")
    calls = {"n": 0}

    def bug():
        calls["n"] += 1
        raise TypeError("a bug, not a host-side failure")

    with pytest.raises(TypeError):
        T_._with_retry(bug, "unit")
    assert calls["n"] == 1

    calls["n"] = 0

    def io_then_ok():
        calls["n"] += 1
        if calls["n"] == 1:
            raise OSError("injected I/O failure")
        return "ok"

    assert T_._with_retry(io_then_ok, "unit") == "ok" and calls["n"] == 2

    calls["n"] = 0
    monkeypatch.setattr(T_, "_device_usable", lambda: False)
    with pytest.raises(OSError):
        T_._with_retry(io_then_ok, "unit")
    assert calls["n"] == 1
