"""Drop-in for the ``eegnet_repl.train`` CLI (PraKesEy/EEGNetReplication src/eegnet_repl/train.py).

    python -m eegnetreplication_amd.train --trainingType Within-Subject --epochs 500
    torchrun --nproc-per-node 8 -m eegnetreplication_amd.train --trainingType Cross-Subject

Same protocols, hyper-parameters, checkpoint names and JSON report schema as the reference:

* Within-Subject (train.py:30-148): per subject the Train+Eval sessions are concatenated, split by
  ``KFold(4, shuffle=True, random_state=42)``; the first ``len(train_val)//5`` of each train_val
  split is validation; EEGNet(p=0.5), Adam(lr=1e-3, eps=1e-7), CE, ``train()``; the best fold by
  validation accuracy is saved as ``models/subject_XX_best_model.pth``.
* Cross-Subject (train.py:151-291): 9 test subjects x 10 repeats = 90 folds; fold k draws
  ``RandomState(42 + k).permutation(other subjects)`` -> 5 train / 3 val subjects; test on the
  subject's Eval session; p=0.25; the fold with the lowest validation loss is saved as
  ``models/cross_subject_best_model.pth``.

MI355X specifics: the folds are independent units, dealt to ranks (one process per GPU) by
``distributed.lpt_assign`` with no communication on the data path and merged on the host; every
split lives in HBM (``DeviceLoader``); each unit is seeded (``--seed`` + unit index), which the
reference does not do, and a fold-indexed launch splits a fold's batch over workgroups by
the batch size alone, so results do not depend on how units are sharded or batched
(tests/test_gpu_sharding.py).  A unit that fails on the host is re-run once from a fresh state.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
from datetime import datetime

import numpy as np
import torch
import torch.nn as nn
from sklearn.model_selection import KFold

from . import distributed as D
from .dataset import BCICI2ADataset, DeviceLoader, build_dataset_from_preprocessed
from .model import EEGNet, evaluate_model, train

logger = logging.getLogger("eegnet_repl")

BATCH_SIZE = 64
EPOCHS = 500
LEARNING_RATE = 0.001
N_SUBJECTS = 9


def _optimizer(model):
    return torch.optim.Adam(model.parameters(), lr=LEARNING_RATE, eps=1e-07, foreach=None, fused=None)


def _run_fold(X, y, tr_ids, va_ids, te, p, epochs, seed, device):
    """One independent unit: build, train, evaluate.  Returns a picklable result dict."""
    torch.manual_seed(seed)
    gen = torch.Generator().manual_seed(seed)
    tl = DeviceLoader(X[tr_ids], y[tr_ids], BATCH_SIZE, shuffle=True, device=device, generator=gen)
    vl = DeviceLoader(X[va_ids], y[va_ids], BATCH_SIZE, shuffle=False, device=device)
    tel = DeviceLoader(te[0], te[1], BATCH_SIZE, shuffle=False, device=device)
    model = EEGNet(C=X.shape[1], T=X.shape[2], p=p)
    opt = _optimizer(model)
    best, _, val_losses, val_accs = train(model, opt, nn.CrossEntropyLoss(), tl, vl, nepochs=epochs)
    model.load_state_dict(best)
    test_acc = evaluate_model(model, tel)
    return {"test_acc": test_acc, "val_acc": max(val_accs), "val_loss": min(val_losses),
            "state": {k: v.detach().cpu() for k, v in best.items()}}


def _run_folds(specs, epochs, device):
    """Several independent units trained together by FoldBatch:
    per-fold streams, one captured hipGraph per fold epoch, no host sync until the end.  Each
    spec is _run_fold's arguments (X, y, tr_ids, va_ids, te, p, seed).  Per fold and epoch, as in
    train() (model.py:101-189): the train loss is the mean of the batch losses, the validation
    loss the mean of per-batch CE means over batches of 64, the validation accuracy over all
    validation trials; the returned state is the final weights (the reference's aliasing "best",
    SURVEY F4).  Returns one result dict per spec, like _run_fold."""
    import torch.nn.functional as F
    from .folds import FoldBatch
    models, seeds, train_sets, val_sets, test_sets, gens = [], [], [], [], [], []
    for X, y, tr_ids, va_ids, te, p, seed in specs:
        torch.manual_seed(seed)
        models.append(EEGNet(C=X.shape[1], T=X.shape[2], p=p).to(device))
        seeds.append(seed)
        gens.append(torch.Generator().manual_seed(seed))

        def dev(a, dt):
            return torch.as_tensor(np.asarray(a), dtype=dt).to(device)
        train_sets.append((dev(X[tr_ids], torch.float32), dev(y[tr_ids], torch.int64)))
        val_sets.append((dev(X[va_ids], torch.float32), dev(y[va_ids], torch.int64)))
        test_sets.append((dev(te[0], torch.float32), dev(te[1], torch.int64)))
    fb = FoldBatch(models, seeds, graphs=True)
    val_loss = [[] for _ in specs]
    val_acc = [[] for _ in specs]
    # validation in groups of folds with the same validation size: one eval launch per fold, then
    # one set of loss / accuracy reductions per group instead of per fold
    groups = {}
    for k, (_, yv) in enumerate(val_sets):
        groups.setdefault(len(yv), []).append(k)
    vgroups = []
    for nv, ks in groups.items():
        nb = (nv + BATCH_SIZE - 1) // BATCH_SIZE
        seg = torch.arange(nv, device=device) // BATCH_SIZE
        vgroups.append((ks, nb, seg, torch.bincount(seg, minlength=nb).double(),
                        torch.stack([val_sets[k][1] for k in ks])))
    for e in range(1, epochs + 1):
        fb.epoch(train_sets, BATCH_SIZE, gens)
        with torch.no_grad():
            logits = []
            for m, (Xv, _) in zip(models, val_sets):
                m.eval()
                logits.append(m(Xv))                # eval BN: batch-size independent
                m.train()
            for ks, nb, seg, cnt, Y in vgroups:
                L = torch.stack([logits[k] for k in ks])                      # [G, nv, classes]
                ce = F.cross_entropy(L.flatten(0, 1), Y.flatten(), reduction="none").view(Y.shape)
                means = torch.zeros((len(ks), nb), dtype=torch.float64, device=ce.device).index_add_(
                    1, seg, ce.double()) / cnt
                vl = means.mean(1)
                va = (L.argmax(2) == Y).sum(1)
                for j, k in enumerate(ks):
                    val_loss[k].append(vl[j])
                    val_acc[k].append(va[j])
        if e == 1 or e % 50 == 0 or e == epochs:
            logger.info(f"Epoch: {e}/{epochs} ({len(specs)} folds batched)")
    out = []
    for k, m in enumerate(models):
        m.eval()
        Xt, yt = test_sets[k]
        with torch.no_grad():
            correct = int((m(Xt).argmax(1) == yt).sum().item())
        vl = torch.stack(val_loss[k]).cpu().numpy()
        va = 100.0 * torch.stack(val_acc[k]).cpu().numpy() / len(val_sets[k][1])
        out.append({"test_acc": 100 * correct / len(yt), "val_acc": float(va.max()),
                    "val_loss": float(vl.min()),
                    "state": {n: v.detach().cpu() for n, v in m.state_dict().items()}})
    return out


UNIT_RETRIES = 1


def _device_fault(e: BaseException) -> bool:
    """A failure of the device itself (HIP error, fault): the context is unusable, so the unit is
    not retried -- the process exits non-zero and the driver re-runs it."""
    msg = str(e)
    return isinstance(e, getattr(torch, "AcceleratorError", ())) or "HIP error" in msg or "CUDA error" in msg


# host-side failures a fresh re-run can cure (I/O, data, host memory); programming errors (TypeError,
# AttributeError, ...) and device faults are not retried
RETRYABLE = (OSError, ValueError, KeyError, IndexError, MemoryError, RuntimeError)


def _device_usable() -> bool:
    """After a failed unit: no stream left in graph capture and the device still synchronises (a
    failure inside torch.cuda.graph capture can leave the stream capturing or invalidated; a re-run
    on it would fail with an unrelated error)."""
    if not torch.cuda.is_available():
        return True
    try:
        if torch.cuda.is_current_stream_capturing():
            return False
        torch.cuda.synchronize()
    except Exception:                                # noqa: BLE001 -- any failure: not usable
        return False
    return True


def _with_retry(fn, what, retries=None):
    """Run one idempotent unit (a fold, or a batch of folds), re-running it from a fresh state if a
    host-side exception escapes (a fold is an idempotent unit).  Every unit builds its
    model, generator and loaders from its own seed, so a re-run reproduces the result bit for bit.
    Only RETRYABLE exceptions that are not device faults are re-run, and only on a device that is
    out of graph capture and still synchronises."""
    retries = UNIT_RETRIES if retries is None else retries
    for attempt in range(retries + 1):
        try:
            return fn()
        except Exception as e:                       # noqa: BLE001 -- re-raised below
            if (attempt == retries or _device_fault(e) or not isinstance(e, RETRYABLE)
                    or not _device_usable()):
                raise
            logger.warning(f"{what} failed ({e!r}); re-running it from a fresh state "
                           f"(attempt {attempt + 2}/{retries + 1})")
    raise AssertionError("unreachable")


def _run_units(specs, epochs, device, fold_batch):
    """Run unit specs one by one (_run_fold) or fold_batch at a time (_run_folds), each unit (or
    fold batch) retried once from a fresh state on a host-side failure."""
    if fold_batch <= 1:
        return [_with_retry(lambda sp=sp: _run_fold(*sp[:5], sp[5], epochs, sp[6], device), f"unit {i}")
                for i, sp in enumerate(specs)]
    # balanced batches of at most fold_batch units (90 cross-subject folds at 48: 45 + 45, not 48 + 42):
    # one fold-indexed launch per pass serves a whole batch, so its size sets the launch width
    nb = -(-len(specs) // fold_batch)
    size = -(-len(specs) // nb) if nb else 0
    res = []
    for i in range(0, len(specs), max(size, 1)):
        batch = specs[i:i + size]
        res.extend(_with_retry(lambda b=batch: _run_folds(b, epochs, device),
                               f"fold batch of units {i}..{i + len(batch) - 1}"))
    return res


def within_subject_units():
    units = []
    for s in range(1, N_SUBJECTS + 1):
        for f in range(4):
            units.append((s, f))
    return units


def _select(units, max_units, world, rank):
    """This rank's unit indices: all units (or the first ``max_units``, a smoke-test restriction
    the reference does not have), dealt by LPT over the ranks."""
    n = len(units) if not max_units else min(int(max_units), len(units))
    return D.lpt_assign([1.0] * n, world)[rank] if world > 1 else list(range(n))


def within_subject_training(epochs=EPOCHS, seed=0, device="cuda", fold_batch=0, max_units=None):
    """train.py:30-148.  Returns (per_subject_test_acc, avg_test_acc, best_model_states).
    ``fold_batch`` > 1 trains that many of this rank's units together (FoldBatch).
    ``max_units`` restricts the run to the first units (subjects with no unit are left out)."""
    rank, world, _ = D.env_rank_world()
    units = within_subject_units()
    mine = _select(units, max_units, world, rank)
    cache, local, specs = {}, {}, []
    for u in mine:
        s, f = units[u]
        if s not in cache:
            tr = build_dataset_from_preprocessed(subject=s)
            ev = build_dataset_from_preprocessed(subject=s, mode="Eval")
            data = BCICI2ADataset(np.concatenate([tr.X, ev.X]), np.concatenate([tr.y, ev.y]))
            splits = list(KFold(n_splits=4, shuffle=True, random_state=42).split(data.X))
            cache[s] = (data, splits)
        data, splits = cache[s]
        train_val, test_ids = splits[f]
        nval = len(train_val) // 5
        logger.info(f"Subject {s} fold {f + 1}/4 on rank {rank}")
        specs.append((data.X, data.y, train_val[nval:], train_val[:nval],
                      (data.X[test_ids], data.y[test_ids]), 0.5, seed + u))
    for u, r in zip(mine, _run_units(specs, epochs, device, fold_batch)):
        local[u] = r
    res = D.gather_results(local)
    per_subject, states = [], []
    for s in range(1, N_SUBJECTS + 1):
        accs, best_val, best_state = [], 0, None
        for f in range(4):
            if units.index((s, f)) not in res:
                continue
            r = res[units.index((s, f))]
            logger.info(f"Subject {s} fold {f + 1}: val {r['val_acc']:.2f}% test {r['test_acc']:.2f}%")
            accs.append(r["test_acc"])
            if r["val_acc"] > best_val:
                best_val, best_state = r["val_acc"], r["state"]
        if not accs:
            continue
        per_subject.append(sum(accs) / len(accs))
        states.append(best_state)
    avg = sum(per_subject) / len(per_subject)
    logger.info(f"Overall Average Test Accuracy across all subjects: {avg:.2f}%")
    return per_subject, avg, states


def cross_subject_units():
    units, k = [], 0
    for s in range(1, N_SUBJECTS + 1):
        others = [o for o in range(1, N_SUBJECTS + 1) if o != s]
        for _ in range(10):
            k += 1
            perm = np.random.RandomState(42 + k).permutation(others)
            units.append((s, k, [int(v) for v in perm[:5]], [int(v) for v in perm[5:]]))
    return units


def cross_subject_training(epochs=EPOCHS, seed=0, device="cuda", fold_batch=0, max_units=None,
                           units_out=None):
    """train.py:151-291.  Returns (best_model_state, per_subject_test_acc, avg_test_acc).
    ``fold_batch`` > 1 trains that many of this rank's folds together (FoldBatch).
    ``max_units`` restricts the run to the first folds (subjects with no fold are left out).
    ``units_out``: a dict that receives every fold's merged result (fold index -> test / validation
    accuracy, validation loss, final state), on every rank."""
    rank, world, _ = D.env_rank_world()
    units = cross_subject_units()
    mine = _select(units, max_units, world, rank)
    sessions = {}

    def sess(s, mode):
        if (s, mode) not in sessions:
            sessions[(s, mode)] = build_dataset_from_preprocessed(subject=s, mode=mode)
        return sessions[(s, mode)]

    local, specs = {}, []
    for u in mine:
        s, k, trs, vas = units[u]
        X = np.concatenate([sess(v, "Train").X for v in trs + vas])
        y = np.concatenate([sess(v, "Train").y for v in trs + vas])
        ntr = sum(len(sess(v, "Train").y) for v in trs)
        ids = np.arange(len(y))
        te = sess(s, "Eval")
        logger.info(f"Fold {k}/90 (Subject {s}) on rank {rank}")
        specs.append((X, y, ids[:ntr], ids[ntr:], (te.X, te.y), 0.25, seed + u))
    for u, r in zip(mine, _run_units(specs, epochs, device, fold_batch)):
        local[u] = r
    res = D.gather_results(local)
    if units_out is not None:
        units_out.update(res)
    per_subject, all_acc = [], []
    best_loss, best_state = 100, None
    for s in range(1, N_SUBJECTS + 1):
        accs = []
        for u, unit in enumerate(units):
            if unit[0] != s or u not in res:
                continue
            r = res[u]
            accs.append(r["test_acc"])
            all_acc.append(r["test_acc"])
            if r["val_loss"] < best_loss:
                best_loss, best_state = r["val_loss"], r["state"]
        if accs:
            per_subject.append(sum(accs) / len(accs))
    avg = sum(all_acc) / len(all_acc)
    se = float(np.std(all_acc) / np.sqrt(len(all_acc)))
    logger.info(f"Overall Average Test Accuracy: {avg:.2f}% +- {se:.2f}%")
    return best_state, per_subject, avg


def _ranked(per_subject, key):
    rows = [{key: i + 1, "test_accuracy": round(a, 2), "performance_rank": 0}
            for i, a in enumerate(per_subject)]
    for rank, r in enumerate(sorted(rows, key=lambda r: r["test_accuracy"], reverse=True), 1):
        r["performance_rank"] = rank
    return rows


def _summary(per_subject, avg):
    return {
        "accuracy_distribution": {
            "above_average_subjects": sum(a > avg for a in per_subject),
            "below_average_subjects": sum(a < avg for a in per_subject),
            "at_average_subjects": sum(a == avg for a in per_subject)},
        "accuracy_quartiles": {
            "q1": round(float(np.percentile(per_subject, 25)), 2),
            "q2_median": round(float(np.percentile(per_subject, 50)), 2),
            "q3": round(float(np.percentile(per_subject, 75)), 2)},
    }


def _mark_data_source(report):
    """Reports trained on seeded synthetic sessions say so (the reference schema is unchanged for
    real data)."""
    from .dataset import synthetic_enabled
    if synthetic_enabled():
        report["data_source"] = "synthetic SMR-like sessions (EEGNET_SYNTHETIC=1), not BCI IV-2a"


def _write_report(report, prefix, out_dir):
    os.makedirs(out_dir, exist_ok=True)
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    path = os.path.join(out_dir, f"{prefix}_training_report_{stamp}.json")
    for p in (path, os.path.join(out_dir, f"latest_{prefix}_report.json")):
        with open(p, "w", encoding="utf-8") as f:
            json.dump(report, f, indent=2, ensure_ascii=False)
    logger.info(f"report written to {path}")
    return path


def generate_ws_report(per_subject_test_acc, avg, states, out_dir="reports"):
    """JSON schema of train.py:309-368."""
    rows = _ranked(per_subject_test_acc, "subject_id")
    for r in rows:
        r["model_saved"] = f"subject_{r['subject_id']:02d}_best_model.pth"
        r["performance_rank"] = r.pop("performance_rank")
    report = {
        "training_type": "Within-Subject",
        "timestamp": datetime.now().isoformat(),
        "model_parameters": {"batch_size": BATCH_SIZE, "epochs": EPOCHS, "learning_rate": LEARNING_RATE,
                             "dropout_probability": 0.5, "cross_validation_folds": 4},
        "overall_results": {"average_test_accuracy": round(avg, 2),
                            "number_of_subjects": len(per_subject_test_acc),
                            "best_subject_accuracy": round(max(per_subject_test_acc), 2),
                            "worst_subject_accuracy": round(min(per_subject_test_acc), 2),
                            "accuracy_std": round(float(np.std(per_subject_test_acc)), 2)},
        "per_subject_results": rows,
        "model_info": {"architecture": "EEGNet", "optimizer": "Adam",
                       "loss_function": "CrossEntropyLoss", "saved_models_count": len(states)},
        "summary_statistics": _summary(per_subject_test_acc, avg),
    }
    _mark_data_source(report)
    return _write_report(report, "within_subject", out_dir)


def generate_cs_report(best_state, per_subject_test_acc, avg, out_dir="reports"):
    """JSON schema of train.py:406-468 (standard_error over per-subject means, as the reference)."""
    report = {
        "training_type": "Cross-Subject",
        "timestamp": datetime.now().isoformat(),
        "model_parameters": {"batch_size": BATCH_SIZE, "epochs": EPOCHS, "learning_rate": LEARNING_RATE,
                             "dropout_probability": 0.25, "total_folds": 90, "repeats_per_subject": 10,
                             "train_subjects_per_fold": 5, "validation_subjects_per_fold": 3},
        "overall_results": {
            "average_test_accuracy": round(avg, 2),
            "standard_error": round(float(np.std(per_subject_test_acc) / np.sqrt(len(per_subject_test_acc))), 2),
            "number_of_test_subjects": len(per_subject_test_acc),
            "best_subject_accuracy": round(max(per_subject_test_acc), 2),
            "worst_subject_accuracy": round(min(per_subject_test_acc), 2),
            "accuracy_std": round(float(np.std(per_subject_test_acc)), 2)},
        "per_subject_results": _ranked(per_subject_test_acc, "test_subject_id"),
        "model_info": {"architecture": "EEGNet", "optimizer": "Adam",
                       "loss_function": "CrossEntropyLoss", "saved_model": "cross_subject_best_model.pth"},
        "summary_statistics": _summary(per_subject_test_acc, avg),
    }
    _mark_data_source(report)
    return _write_report(report, "cross_subject", out_dir)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="Train a EEGNet model (MI355X).")
    ap.add_argument("--trainingType", type=str, default="Within-Subject",
                    help="Training type [Cross-Subject, Within-Subject].")
    ap.add_argument("--epochs", type=int, default=EPOCHS, help="Number of training epochs.")
    ap.add_argument("--generateReport", type=bool, default=True, help="Generate report after training.")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", type=str, default=".", help="directory for models/ and reports/")
    ap.add_argument("--fold-batch", type=int, default=90,
                    help="train up to this many folds together on one GPU (FoldBatch, balanced batches); "
                         "0/1: one at a time")
    ap.add_argument("--max-units", type=int, default=0,
                    help="smoke runs: only the first N folds of the protocol (0 = all)")
    ap.add_argument("--synthetic", action="store_true",
                    help="train on seeded synthetic sessions when data/processed/*.npz is absent "
                         "(same as EEGNET_SYNTHETIC=1); the reports record it")
    args = ap.parse_args(argv)
    if args.synthetic:
        os.environ["EEGNET_SYNTHETIC"] = "1"
    logging.basicConfig(level=logging.INFO,
                        format="%(asctime)s - %(filename)s - %(funcName)s - %(levelname)s - %(message)s",
                        handlers=[logging.FileHandler("app.log"), logging.StreamHandler()])
    rank, world, local = D.init_process_group()
    device = f"cuda:{local}"
    torch.cuda.set_device(local)
    models_dir = os.path.join(args.out, "models")
    reports_dir = os.path.join(args.out, "reports")
    if args.trainingType == "Within-Subject":
        per_subject, avg, states = within_subject_training(args.epochs, args.seed, device, args.fold_batch,
                                                           args.max_units)
        if rank == 0:
            os.makedirs(models_dir, exist_ok=True)
            for s, st in enumerate(states, 1):        # train.py:136-139 (max_units keeps 1..k)
                torch.save(st, os.path.join(models_dir, f"subject_{s:02d}_best_model.pth"))
            if args.generateReport:
                generate_ws_report(per_subject, avg, states, reports_dir)
    else:
        best, per_subject, avg = cross_subject_training(args.epochs, args.seed, device, args.fold_batch,
                                                        args.max_units)
        if rank == 0:
            os.makedirs(models_dir, exist_ok=True)
            torch.save(best, os.path.join(models_dir, "cross_subject_best_model.pth"))
            if args.generateReport:
                generate_cs_report(best, per_subject, avg, reports_dir)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
