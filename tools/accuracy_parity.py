"""Accuracy parity (north_star: "accuracy within +-1 pt over fixed seeds").

The within-subject protocol (train.py:30-148: 9 subjects x 4 KFold folds, batch 64, Adam(1e-3,
eps 1e-7), CE, p = 0.5, final weights, test accuracy in eval mode) is run twice on the
seeded synthetic SMR sessions (eegnetreplication_amd.dataset.synthetic_session; real BCI IV-2a data
is absent):

* HIP: the product path (train._run_units, FoldBatch + the fused HIP step);
* reference: the reference's layer stack on stock ATen ops (oracle/torch_ref.py, fp32, on the same
  device), trained by a restatement of model.py:101-189 -- same splits, same initial weights (the
  same torch.manual_seed(seed) before EEGNet()), same batch order (DataLoader's generator
  consumption, dataset.epoch_permutation); dropout masks come from torch's RNG (nn.Dropout) and
  from the device generator respectively, so the comparison is statistical for p > 0.

    python tools/accuracy_parity.py --epochs 100 --seeds 0 1 2 [--p 0.5] [--out file.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def unit_specs(seed, p):
    from sklearn.model_selection import KFold
    from eegnetreplication_amd.dataset import synthetic_session
    from eegnetreplication_amd.train import within_subject_units
    specs, cache = [], {}
    for u, (s, f) in enumerate(within_subject_units()):
        if s not in cache:
            tr, ev = synthetic_session(s, "Train"), synthetic_session(s, "Eval")
            X = np.concatenate([tr.X, ev.X])
            y = np.concatenate([tr.y, ev.y])
            cache[s] = (X, y, list(KFold(n_splits=4, shuffle=True, random_state=42).split(X)))
        X, y, splits = cache[s]
        tv, te = splits[f]
        nval = len(tv) // 5
        specs.append((X, y, tv[nval:], tv[:nval], (X[te], y[te]), p, seed + u))
    return specs


def run_reference(spec, epochs, dev):
    """model.py:101-189 + evaluate_model on the stock-ATen restatement (fp32, dropout by torch)."""
    from eegnetreplication_amd.dataset import epoch_permutation
    from eegnetreplication_amd.model import EEGNet
    from oracle import torch_ref as tr
    X, y, tr_ids, va_ids, te, p, seed = spec
    torch.manual_seed(seed)
    init = EEGNet(C=X.shape[1], T=X.shape[2], p=p)
    ref = tr.TorchRefEEGNet({k: v.numpy() for k, v in init.state_dict().items()}, p=p, device=dev)
    opt = tr.make_optimizer(ref)
    gen = torch.Generator().manual_seed(seed)
    Xt = torch.as_tensor(X[tr_ids], dtype=torch.float32, device=dev)
    yt = torch.as_tensor(y[tr_ids], dtype=torch.int64, device=dev)
    for _ in range(epochs):
        ref.training = True
        perm = epoch_permutation(len(yt), gen).to(dev)
        for i in range(0, len(yt), 64):
            idx = perm[i:i + 64]
            tr.train_step(ref, opt, Xt.index_select(0, idx), yt.index_select(0, idx))
    ref.training = False                     # train() leaves the model in eval mode (model.py:151)
    with torch.no_grad():
        out = ref(torch.as_tensor(te[0], dtype=torch.float32, device=dev))
    return 100.0 * float((out.argmax(1).cpu() == torch.as_tensor(te[1])).float().mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--p", type=float, default=0.5)
    ap.add_argument("--fold-batch", type=int, default=36)
    ap.add_argument("--out", type=str, default="")
    args = ap.parse_args()
    from eegnetreplication_amd.train import _run_units
    dev = torch.device("cuda:0")
    res = {"protocol": "within-subject (train.py:30-148) on seeded synthetic SMR sessions",
           "epochs": args.epochs, "p": args.p, "seeds": args.seeds, "runs": []}
    for seed in args.seeds:
        specs = unit_specs(seed, args.p)
        t0 = time.perf_counter()
        hip = [r["test_acc"] for r in _run_units(specs, args.epochs, dev, args.fold_batch)]
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ref = []
        for i, sp in enumerate(specs):
            ref.append(run_reference(sp, args.epochs, dev))
            if i % 6 == 5:
                print(f"  seed {seed}: reference unit {i + 1}/{len(specs)} "
                      f"({time.perf_counter() - t1:.0f} s)", flush=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        run = {"seed": seed, "hip_mean": float(np.mean(hip)), "ref_mean": float(np.mean(ref)),
               "hip": hip, "ref": ref, "hip_s": round(t1 - t0, 1), "ref_s": round(t2 - t1, 1)}
        res["runs"].append(run)
        print(f"seed {seed}: HIP {run['hip_mean']:.2f}%  reference {run['ref_mean']:.2f}%  "
              f"({run['hip_s']} s / {run['ref_s']} s)", flush=True)
    h = np.array([np.mean(r["hip"]) for r in res["runs"]])
    f = np.array([np.mean(r["ref"]) for r in res["runs"]])
    allh = np.concatenate([r["hip"] for r in res["runs"]])
    allf = np.concatenate([r["ref"] for r in res["runs"]])
    res["hip_mean"], res["ref_mean"] = float(allh.mean()), float(allf.mean())
    res["diff_pt"] = float(allh.mean() - allf.mean())
    # standard error of the mean paired difference (same unit, split, init and batch order; the
    # dropout masks differ)
    d = allh - allf
    res["diff_se_pt"] = float(d.std(ddof=1) / np.sqrt(len(d)))
    res["per_seed_diff_pt"] = [float(a - b) for a, b in zip(h, f)]
    print(json.dumps({k: v for k, v in res.items() if k != "runs"}), flush=True)
    if args.out:
        with open(args.out, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
