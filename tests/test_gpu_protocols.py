"""The protocol layer on the GPU (cfg1 / cfg3 callers):

* the CLI ``python -m eegnet_repl.train`` end to end on the seeded synthetic sessions, for both
  protocols, one fold at a time (``--fold-batch 0``) and fold-batched (``--fold-batch 16``):
  checkpoint and report file names and schema (train.py:136-139, 286-289, 309-468), and every saved
  ``.pth`` loads with ``map_location='cpu'`` into a reference-shaped module the way the reference's
  UI loads it (ui.py:26-36) and evaluates there, on the CPU, to the logits the HIP eval kernel gives;
* ``train()`` (model.py:101-189) over whole epochs -- device-resident shuffled loader, fused and
  autograd paths -- against a float64 oracle loop over the same batches.
"""

from __future__ import annotations

import glob
import json
import os

import numpy as np
import pytest
import torch
import torch.nn as nn

from golden_util import PARAM_NAMES, assert_close, assert_params_close

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


WS_KEYS = {"training_type", "timestamp", "model_parameters", "overall_results",
           "per_subject_results", "model_info", "summary_statistics", "data_source"}


def _load_like_ui(path):
    """ui.py:26-36: torch.load(map_location='cpu') into EEGNet(22, 256); here through safe loading
    (weights_only=True) into (a) this build's module, built on the CPU, and (b) the reference layer
    stack restated with stock ATen ops (oracle/torch_ref.py), which then evaluates on the CPU."""
    from eegnet_repl.model import EEGNet
    from oracle import torch_ref as tr
    sd = torch.load(path, map_location="cpu", weights_only=True)
    m = EEGNet(22, 256)
    m.load_state_dict(sd)
    ref = tr.TorchRefEEGNet({k: v.numpy() for k, v in sd.items()}, p=0.5)
    ref.training = False
    return sd, m, ref


def _check_checkpoint(path, dev):
    sd, m, ref = _load_like_ui(path)
    assert len(sd) == 21 and int(sd["temporal.1.num_batches_tracked"]) > 0
    x = torch.from_numpy(np.random.default_rng(1).standard_normal((6, 22, 256)).astype(np.float32))
    with torch.no_grad():
        cpu_logits = ref(x).numpy()
    m = m.to(dev).eval()
    with torch.no_grad():
        gpu_logits = m(x.to(dev)).cpu().numpy()
    assert_close(gpu_logits, cpu_logits, rtol=1e-4, atol_frac=1e-5, name=os.path.basename(path))


@pytest.mark.parametrize("fold_batch", [0, 16])
def test_cli_within_subject_end_to_end(tmp_path, monkeypatch, fold_batch):
    from eegnet_repl import train as cli
    dev = _dev()
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("EEGNET_DATA_DIR", str(tmp_path / "nodata"))
    cli.main(["--trainingType", "Within-Subject", "--epochs", "2", "--synthetic",
              "--fold-batch", str(fold_batch), "--out", str(tmp_path)])
    models = sorted(os.path.basename(p) for p in glob.glob(str(tmp_path / "models" / "*.pth")))
    assert models == [f"subject_{s:02d}_best_model.pth" for s in range(1, 10)]
    reps = glob.glob(str(tmp_path / "reports" / "within_subject_training_report_*.json"))
    assert len(reps) == 1
    r = json.load(open(tmp_path / "reports" / "latest_within_subject_report.json"))
    assert set(r) == WS_KEYS and r["training_type"] == "Within-Subject"
    assert r["model_parameters"]["cross_validation_folds"] == 4
    assert len(r["per_subject_results"]) == 9
    assert sorted(x["performance_rank"] for x in r["per_subject_results"]) == list(range(1, 10))
    assert 0.0 <= r["overall_results"]["average_test_accuracy"] <= 100.0
    assert "synthetic" in r["data_source"]
    for p in (1, 9):
        _check_checkpoint(str(tmp_path / "models" / f"subject_{p:02d}_best_model.pth"), dev)


@pytest.mark.parametrize("fold_batch", [0, 16])
def test_cli_cross_subject_end_to_end(tmp_path, monkeypatch, fold_batch):
    """The first 12 of the 90 folds (subject 1's ten repeats, subject 2's first two)."""
    from eegnet_repl import train as cli
    dev = _dev()
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("EEGNET_DATA_DIR", str(tmp_path / "nodata"))
    cli.main(["--trainingType", "Cross-Subject", "--epochs", "2", "--synthetic", "--max-units", "12",
              "--fold-batch", str(fold_batch), "--out", str(tmp_path)])
    assert os.path.exists(tmp_path / "models" / "cross_subject_best_model.pth")
    r = json.load(open(tmp_path / "reports" / "latest_cross_subject_report.json"))
    assert r["training_type"] == "Cross-Subject"
    assert r["model_parameters"]["total_folds"] == 90
    assert r["model_parameters"]["dropout_probability"] == 0.25
    assert [x["test_subject_id"] for x in r["per_subject_results"]] == [1, 2]
    assert r["model_info"]["saved_model"] == "cross_subject_best_model.pth"
    _check_checkpoint(str(tmp_path / "models" / "cross_subject_best_model.pth"), dev)


def test_cli_refuses_missing_data_without_synthetic(tmp_path, monkeypatch):
    from eegnet_repl import train as cli
    _dev()
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("EEGNET_DATA_DIR", str(tmp_path / "nodata"))
    monkeypatch.delenv("EEGNET_SYNTHETIC", raising=False)
    with pytest.raises(ValueError, match="No preprocessed files"):
        cli.main(["--trainingType", "Within-Subject", "--epochs", "1", "--out", str(tmp_path)])


# ---------------------------------------------------------------------------------------------
# train() over epochs vs a float64 oracle loop
# ---------------------------------------------------------------------------------------------
def _oracle_train(params, bufs, X, y, Xv, yv, epochs, seed):
    """model.py:101-189 restated on the numpy oracle: per epoch, batches of 64 in the DataLoader
    order for generator seed ``seed`` (dataset.epoch_permutation), forward/CE/backward/clamps/Adam;
    validation in eval mode over batches of 64 (mean of batch CE means, accuracy)."""
    from eegnetreplication_amd.dataset import epoch_permutation
    from oracle import numpy_ref as nr
    st = nr.adam_init(params)
    g = torch.Generator().manual_seed(seed)
    tl, vl, va = [], [], []
    for _ in range(epochs):
        perm = epoch_permutation(len(y), g).numpy()
        losses = []
        for i in range(0, len(y), 64):
            idx = perm[i:i + 64]
            out = nr.train_step(params, bufs, X[idx], y[idx], st, p=0.0)
            params, bufs = out["params"], out["buffers"]
            losses.append(out["loss"])
        tl.append(float(np.mean(losses)))
        vls, correct = [], 0
        for i in range(0, len(yv), 64):
            lg, _, _ = nr.forward(params, bufs, Xv[i:i + 64], train=False)
            vls.append(nr.cross_entropy(lg, yv[i:i + 64])[0])
            correct += int((lg.argmax(1) == yv[i:i + 64]).sum())
        vl.append(float(np.mean(vls)))
        va.append(100 * correct / len(yv))
    return params, bufs, tl, vl, va


@pytest.mark.parametrize("fused", [True, False])
def test_train_loop_matches_oracle_over_epochs(fused):
    """3 epochs of train() on 150 trials of 22 x 257 (p = 0, batch 64 with a short last batch,
    shuffled by a seeded generator) + validation every epoch: final weights, BN running statistics,
    per-epoch train/val losses and val accuracies against the float64 oracle on the same batches.
    fused=True: one device sequence per step; fused=False: autograd through the HIP kernels and
    torch.optim.Adam (foreach on the device)."""
    from eegnetreplication_amd.dataset import DeviceLoader
    from eegnetreplication_amd.model import EEGNet, train
    dev = _dev()
    rng = np.random.default_rng(21)
    X = rng.standard_normal((150, 22, 257))
    y = rng.integers(0, 4, 150).astype(np.int64)
    Xv = rng.standard_normal((70, 22, 257))
    yv = rng.integers(0, 4, 70).astype(np.int64)
    torch.manual_seed(4)
    model = EEGNet(22, 257, p=0.0)
    p0 = {k: v.detach().numpy().copy() for k, v in model.named_parameters()}
    b0 = {k: v.detach().numpy().copy() for k, v in model.named_buffers()}
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, eps=1e-7)
    tl_ = DeviceLoader(X, y, 64, shuffle=True, device=dev, generator=torch.Generator().manual_seed(9))
    vl_ = DeviceLoader(Xv, yv, 64, shuffle=False, device=dev)
    best, tl, vl, va = train(model, opt, nn.CrossEntropyLoss(), tl_, vl_, nepochs=3, fused=fused)
    params, bufs, otl, ovl, ova = _oracle_train(p0, b0, X.astype(np.float32).astype(np.float64), y,
                                               Xv.astype(np.float32).astype(np.float64), yv, 3, 9)
    np.testing.assert_allclose(tl, otl, rtol=2e-4)
    np.testing.assert_allclose(vl, ovl, rtol=2e-4)
    assert va == ova
    assert_params_close({k: p.detach().cpu().numpy() for k, p in model.named_parameters()}, params,
                        steps=9, rtol=2e-4, atol_frac=2e-4)
    # BN1's affine parameters get rounding-residue gradients (golden_util.NEAR_ZERO_GRADS), so Adam
    # moves them by up to ~lr per step with noise signs in either implementation.  The loss cannot
    # see them, but BN2's running statistics do: its batch mean is a1 mean(v) + c1 W with
    # c1 = beta1 - a1 mu1 and W[o] = sum_c ws[o,c], its variance scales with gamma1^2.  Those two
    # buffers are judged with the bound the observed beta1 / gamma1 differences imply.
    hp = {k: p.detach().cpu().numpy().astype(np.float64) for k, p in model.named_parameters()}
    dbeta = float(np.abs(hp["temporal.1.bias"] - params["temporal.1.bias"]).max())
    dgam = float((np.abs(hp["temporal.1.weight"] - params["temporal.1.weight"])
                  / np.abs(params["temporal.1.weight"])).max())
    # The bound cannot calibrate itself past physics: Adam moves an element by <= ~lr per step,
    # so both differences are capped a priori at 2 lr steps (assert_params_close above holds the
    # same cap), whatever the run observed.
    cap = 2 * 1e-3 * 9
    assert dbeta <= cap
    assert float(np.abs(hp["temporal.1.weight"] - params["temporal.1.weight"]).max()) <= cap
    W = float(np.abs(params["spatial.weight"].reshape(16, -1).sum(1)).max())
    for k, b in model.named_buffers():
        got = b.detach().cpu().numpy()
        if "num_batches_tracked" in k:
            assert int(b) == 9 and int(best[k]) == 9        # F4: "best" aliases the live state
        elif k == "aggregation.0.running_mean":
            assert_close(got, bufs[k], rtol=2e-4, atol_abs=1e-5 + 2 * dbeta * W, name=k)
        elif k == "aggregation.0.running_var":
            assert_close(got, bufs[k], rtol=2e-4 + 4 * dgam, atol_abs=1e-5, name=k)
        else:
            assert_close(got, bufs[k], rtol=2e-4, atol_abs=1e-5, name=k)
    for k in PARAM_NAMES:                                    # final weights returned
        assert torch.equal(best[k], dict(model.named_parameters())[k].detach())
