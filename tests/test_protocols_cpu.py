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
    blob = json.dumps([[u[2], u[3]] for u in units]).encode()
    assert len(hashlib.sha256(blob).hexdigest()) == 64


def test_synthetic_sessions_shape_and_determinism():
    from eegnetreplication_amd.dataset import build_dataset_from_preprocessed
    a = build_dataset_from_preprocessed(3)
    b = build_dataset_from_preprocessed(3)
    e = build_dataset_from_preprocessed(3, mode="Eval")
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
