"""Accuracy parity (north_star: "BCI IV-2a accuracy within +-1 pt over fixed seeds").

Both protocols of the reference CLI, at the reference's 500 epochs (train.py:26), on the seeded
synthetic SMR sessions (eegnetreplication_amd.dataset.synthetic_session; real BCI IV-2a data is
absent, SURVEY F7 -- real-data parity stays unpinned: the reference's one real-data anchor, subject
3 at 74.31 %, notebooks/07_function_tests.ipynb:343, cannot be reproduced here):

* within-subject (train.py:30-148): 9 subjects x 4 KFold folds, p = 0.5;
* cross-subject (train.py:151-291): a fixed subset of the 90 folds (default: the first two repeats
  of every test subject, 18 folds), p = 0.25.

Each unit (same split, same initial weights -- torch.manual_seed(unit seed) before EEGNet() --, same
batch order -- DataLoader's generator consumption, dataset.epoch_permutation) is trained twice:

* HIP: the product path (train._run_units: FoldBatch, fold-indexed launches, the fused HIP step);
* reference: the reference's layer stack on stock ATen ops (oracle/torch_ref.py, fp32, on the same
  device), trained by a restatement of model.py:101-189, final weights, test accuracy
  in eval mode (model.py:151).

Dropout, two ways (``--dropout``):
* ``independent``: the reference draws its masks from torch's RNG (nn.Dropout semantics), the HIP
  path from its device generator -- the north_star's "over fixed seeds" sense, statistical only;
* ``common``: the reference is given exactly the masks the HIP device generator draws (restated in
  torch below, keyed by (unit seed, step) as eegnet_common.h fold_drop_key / keep_mul), so the two
  runs differ only by fp32 rounding -- common random numbers, a far tighter paired comparison.

Reported per protocol and dropout mode: per-unit paired differences, their mean, standard error,
95 % confidence interval (Student t), and per-seed means.  The reference units run in worker
processes on the one GPU (each regenerates the seeded specs itself).

    python tools/accuracy_parity.py --protocol ws --epochs 500 --seeds 0 1 2 3 4 --dropout common
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

M32 = 0xFFFFFFFF


def ws_specs(seed):
    """within_subject_training's units (train.py:50-89), p = 0.5."""
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
        specs.append((X, y, tv[nval:], tv[:nval], (X[te], y[te]), 0.5, seed + u))
    return specs


def cs_specs(seed, folds):
    """cross_subject_training's folds (train.py:182-231) with the given 0-based fold indices, p = 0.25."""
    from eegnetreplication_amd.dataset import synthetic_session
    from eegnetreplication_amd.train import cross_subject_units
    units = cross_subject_units()
    sess = {}

    def get(s, mode):
        if (s, mode) not in sess:
            sess[(s, mode)] = synthetic_session(s, mode)
        return sess[(s, mode)]

    specs = []
    for u in folds:
        s, k, trs, vas = units[u]
        X = np.concatenate([get(v, "Train").X for v in trs + vas])
        y = np.concatenate([get(v, "Train").y for v in trs + vas])
        ntr = sum(len(get(v, "Train").y) for v in trs)
        ids = np.arange(len(y))
        te = get(s, "Eval")
        specs.append((X, y, ids[:ntr], ids[ntr:], (te.X, te.y), 0.25, seed + u))
    return specs


def specs_for(protocol, seed, cs_folds):
    return ws_specs(seed) if protocol == "ws" else cs_specs(seed, cs_folds)


# ---- the HIP device dropout generator, restated in torch (eegnet_host.hip mix_key, eegnet_common.h
# ---- fold_drop_key / keep_mul; tests/hip_cases.py holds the numpy twin) -------------------------
def mix_key(seed: int, offset: int) -> int:
    m = (1 << 64) - 1
    z = (seed * 0xD1B54A32D192ED03 + offset * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _keep(n: int, key: int, pthr: int, dev) -> torch.Tensor:
    h = torch.arange(n, dtype=torch.int64, device=dev)
    h = (h * 0x9E3779B1 + key) & M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    h = h ^ (h >> 16)
    return (h >> 8) >= pthr


def device_masks(B, F2, T, seed, step, p, dev):
    key = mix_key(seed, step)
    k0, k1 = key & M32, ((key >> 32) ^ 0x5BD1E995) & M32
    pthr = int(min(16777216.0, max(0.0, float(np.float32(p)) * 16777216.0)))
    T1 = T // 4
    T2 = T1 // 8
    return (_keep(B * F2 * T1, k0, pthr, dev).view(B, F2, T1),
            _keep(B * F2 * T2, k1, pthr, dev).view(B, F2, T2))


def run_reference(spec, epochs, dev, common):
    """model.py:101-189 + evaluate_model on the stock-ATen restatement (fp32)."""
    from eegnetreplication_amd.dataset import epoch_permutation
    from oracle import torch_ref as tr
    X, y, tr_ids, va_ids, te, p, seed = spec
    torch.manual_seed(seed)                  # the HIP unit's EEGNet() draws the same initial weights
    init = tr.init_state(C=X.shape[1], T=X.shape[2])
    ref = tr.TorchRefEEGNet({k: v.numpy() for k, v in init.items()}, p=p, device=dev)
    opt = tr.make_optimizer(ref)
    gen = torch.Generator().manual_seed(seed)
    Xt = torch.as_tensor(X[tr_ids], dtype=torch.float32, device=dev)
    yt = torch.as_tensor(y[tr_ids], dtype=torch.int64, device=dev)
    F2, T = init["spatial.weight"].shape[0], X.shape[2]
    step = 0
    for _ in range(epochs):
        ref.training = True
        perm = epoch_permutation(len(yt), gen).to(dev)
        for i in range(0, len(yt), 64):
            idx = perm[i:i + 64]
            masks = device_masks(len(idx), F2, T, seed, step, p, dev) if common and p > 0 else None
            tr.train_step(ref, opt, Xt.index_select(0, idx), yt.index_select(0, idx), masks)
            step += 1
    ref.training = False                     # train() leaves the model in eval mode (model.py:151)
    with torch.no_grad():
        out = ref(torch.as_tensor(te[0], dtype=torch.float32, device=dev))
    return 100.0 * float((out.argmax(1).cpu() == torch.as_tensor(te[1])).float().mean())


def _keep_t(n: int, key: torch.Tensor, pthr: int, dev) -> torch.Tensor:
    """_keep with the 32-bit key a device tensor (graph-capturable: the key is read, not baked in)."""
    h = torch.arange(n, dtype=torch.int64, device=dev)
    h = (h * 0x9E3779B1 + key) & M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    h = h ^ (h >> 16)
    return (h >> 8) >= pthr


def run_reference_graphed(spec, epochs, dev, common):
    """run_reference with each epoch's training steps captured once as a CUDA graph and replayed
    (the reference is launch-bound at batch 64: ~80 small kernels per step).  The same layer stack,
    loss, clamps and batch order; Adam with capturable=True (its bias corrections as device tensors:
    the same formula, rounding-level differences); the common-mask keys of every step precomputed and
    read in the graph through a device step counter; the epoch's permutation copied into the graph's
    static buffer before each replay.  The first epoch runs eagerly (Adam's state is created lazily)."""
    from eegnetreplication_amd.dataset import epoch_permutation
    from oracle import torch_ref as tr
    import torch.nn.functional as F
    X, y, tr_ids, va_ids, te, p, seed = spec
    torch.manual_seed(seed)                  # the HIP unit's EEGNet() draws the same initial weights
    init = tr.init_state(C=X.shape[1], T=X.shape[2])
    ref = tr.TorchRefEEGNet({k: v.numpy() for k, v in init.items()}, p=p, device=dev)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, eps=1e-7, capturable=True)
    gen = torch.Generator().manual_seed(seed)
    Xt = torch.as_tensor(X[tr_ids], dtype=torch.float32, device=dev)
    yt = torch.as_tensor(y[tr_ids], dtype=torch.int64, device=dev)
    n = len(yt)
    F2, T = init["spatial.weight"].shape[0], X.shape[2]
    T1, T2 = T // 4, (T // 4) // 8
    nsteps = -(-n // 64)
    keys = None
    pthr = int(min(16777216.0, max(0.0, float(np.float32(p)) * 16777216.0)))
    if common and p > 0:
        kk = []
        for st in range(epochs * nsteps):
            key = mix_key(seed, st)
            kk.append([key & M32, ((key >> 32) ^ 0x5BD1E995) & M32])
        keys = torch.tensor(kk, dtype=torch.int64, device=dev)
    step_t = torch.zeros(1, dtype=torch.int64, device=dev)
    perm_buf = torch.zeros(n, dtype=torch.int64, device=dev)
    for prm in ref.parameters():
        prm.grad = torch.zeros_like(prm)

    def epoch_body():
        for i in range(0, n, 64):
            idx = perm_buf[i:i + 64]
            B = idx.shape[0]
            masks = None
            if keys is not None:
                kr = keys.index_select(0, step_t)[0]
                masks = (_keep_t(B * F2 * T1, kr[0], pthr, dev).view(B, F2, T1),
                         _keep_t(B * F2 * T2, kr[1], pthr, dev).view(B, F2, T2))
            logits = ref(Xt.index_select(0, idx), masks)
            loss = F.cross_entropy(logits, yt.index_select(0, idx))
            opt.zero_grad(set_to_none=False)
            loss.backward()
            opt.step()
            step_t.add_(1)

    ref.training = True
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    graph = None
    with torch.cuda.stream(s):
        for e in range(epochs):
            perm_buf.copy_(epoch_permutation(n, gen).to(dev))
            if e == 0:
                epoch_body()                         # eager: Adam's state, cuDNN/MIOpen plans
                continue
            if graph is None:
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                saved = step_t.clone()
                with torch.cuda.graph(graph, stream=s):
                    epoch_body()
                step_t.copy_(saved)                  # (capture recorded, did not run)
            graph.replay()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref.training = False                     # train() leaves the model in eval mode (model.py:151)
    with torch.no_grad():
        out = ref(torch.as_tensor(te[0], dtype=torch.float32, device=dev))
    return 100.0 * float((out.argmax(1).cpu() == torch.as_tensor(te[1])).float().mean())


def _hip_lib_mapped() -> bool:
    """Whether this process has libeegnet_hip*.so mapped (/proc/self/maps)."""
    try:
        with open("/proc/self/maps") as f:
            return any("libeegnet_hip" in line for line in f)
    except OSError:
        return False


def _worker(wid, jobs, protocol, cs_folds, epochs, common, q, graphed=True):
    """Reference units (seed, unit index) -> (seed, unit, accuracy); specs regenerated here.

    A reference worker runs stock ATen ops only: its initial weights come from the oracle's
    restatement of the reference's module construction (oracle/torch_ref.init_state), so nothing in
    it imports the product's model or loads libeegnet_hip.so -- checked from /proc/self/maps at start
    and after every unit and reported with each result (round-4 VERDICT item 3)."""
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    q.put(("info", wid, {"maps_lib_at_start": _hip_lib_mapped(), "pid": os.getpid(),
                         "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")}))
    cache = {}
    for seed, u in jobs:
        if seed not in cache:
            cache = {seed: specs_for(protocol, seed, cs_folds)}
        t0 = time.perf_counter()
        acc = (run_reference_graphed if graphed else run_reference)(cache[seed][u], epochs, dev, common)
        q.put((seed, u, acc, time.perf_counter() - t0, _hip_lib_mapped()))


def t_crit_95(df):
    from scipy import stats
    return float(stats.t.ppf(0.975, df))


def summarize(pairs):
    d = np.array([h - r for h, r in pairs], dtype=np.float64)
    n = len(d)
    se = float(d.std(ddof=1) / np.sqrt(n)) if n > 1 else float("nan")
    tc = t_crit_95(n - 1) if n > 1 else float("nan")
    return {"n_pairs": n, "diff_mean_pt": float(d.mean()), "diff_sd_pt": float(d.std(ddof=1)) if n > 1 else 0.0,
            "diff_se_pt": se, "ci95_pt": [float(d.mean() - tc * se), float(d.mean() + tc * se)],
            "pairs_identical": int((d == 0).sum())}


def main():
    import torch.multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--protocol", choices=["ws", "cs"], default="ws")
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3, 4])
    ap.add_argument("--dropout", choices=["independent", "common"], default="common")
    ap.add_argument("--cs-folds", type=int, nargs="+",
                    default=[10 * s + r for s in range(9) for r in range(2)],
                    help="0-based cross-subject fold indices (default: repeats 1-2 of every subject)")
    ap.add_argument("--workers", type=int, default=8, help="reference worker processes on the GPU")
    ap.add_argument("--worker-hw-queues", type=int, default=1,
                    help="GPU_MAX_HW_QUEUES of each reference worker (one stream each: round 4 ran 15 "
                         "workers at HIP's default 4, 60+ user queues on one GPU, and lost one to an "
                         "illegal-instruction fault in a stock fill kernel)")
    ap.add_argument("--ref-eager", action="store_true",
                    help="train the reference units step by step (no CUDA graph; the original driver)")
    ap.add_argument("--out", type=str, default="")
    args = ap.parse_args()
    from eegnetreplication_amd.train import _run_units
    dev = torch.device("cuda:0")
    common = args.dropout == "common"
    res = {"protocol": {"ws": "within-subject (train.py:30-148), p = 0.5",
                        "cs": "cross-subject (train.py:151-291), p = 0.25, folds " + str(args.cs_folds)}[args.protocol],
           "data": "seeded synthetic SMR sessions (dataset.synthetic_session); real BCI IV-2a parity is "
                   "unpinned (anchor: subject 3 at 74.31 %, notebooks/07_function_tests.ipynb:343)",
           "epochs": args.epochs, "seeds": args.seeds, "dropout": args.dropout, "runs": []}
    n_units = 36 if args.protocol == "ws" else len(args.cs_folds)
    jobs = [(s, u) for s in args.seeds for u in range(n_units)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    nw = max(1, min(args.workers, len(jobs)))
    procs = [ctx.Process(target=_worker, args=(w, jobs[w::nw], args.protocol, args.cs_folds, args.epochs,
                                                common, q, not args.ref_eager)) for w in range(nw)]
    t_start = time.perf_counter()
    # the workers inherit the environment at spawn: their HIP runtime reads GPU_MAX_HW_QUEUES at init
    saved_q = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = str(args.worker_hw_queues)
    for p in procs:
        p.start()
    if saved_q is None:
        os.environ.pop("GPU_MAX_HW_QUEUES", None)
    else:
        os.environ["GPU_MAX_HW_QUEUES"] = saved_q
    res["workers"] = nw
    res["worker_hw_queues"] = args.worker_hw_queues
    res["worker_info"] = {}
    hip = {}
    for seed in args.seeds:                   # the HIP units meanwhile, in this process
        specs = specs_for(args.protocol, seed, args.cs_folds)
        t0 = time.perf_counter()
        out = _run_units(specs, args.epochs, dev, len(specs))
        torch.cuda.synchronize()
        hip[seed] = [r["test_acc"] for r in out]
        print(f"seed {seed}: HIP {np.mean(hip[seed]):.2f}% ({time.perf_counter() - t0:.1f} s)", flush=True)
    ref = {}
    import queue as _queue
    import signal

    def _stop(signum, frame):                 # the call's time limit: keep what finished (below)
        signal.signal(signal.SIGTERM, signal.SIG_IGN)   # once: the workers' group may get it too
        raise KeyboardInterrupt
    signal.signal(signal.SIGTERM, _stop)
    args.worker_info = res["worker_info"]
    args.worker_lib_mapped = False
    try:
        _collect(jobs, q, procs, ref, t_start, hip, args)
    except KeyboardInterrupt:
        print(f"  stopped with {len(ref)}/{len(jobs)} reference units: recording those", flush=True)
        for p in procs:
            try:
                p.kill()
            except Exception:                 # already gone
                pass
    res["worker_lib_mapped"] = args.worker_lib_mapped or any(
        i.get("maps_lib_at_start") for i in res["worker_info"].values())
    done_seeds = [sd for sd in args.seeds if all((sd, u) in ref for u in range(n_units))]
    res["complete"] = len(ref) == len(jobs)
    pairs = []
    for seed in args.seeds:
        us = [u for u in range(n_units) if (seed, u) in ref]
        if not us:
            continue
        r = [ref[(seed, u)] for u in us]
        h = [hip[seed][u] for u in us]
        res["runs"].append({"seed": seed, "units": us, "hip": h, "ref": r, "hip_mean": float(np.mean(h)),
                            "ref_mean": float(np.mean(r)), "diff_pt": float(np.mean(h) - np.mean(r))})
        pairs += list(zip(h, r))
    res["complete_seeds"] = done_seeds
    res["hip_mean"] = float(np.mean([h for h, _ in pairs]))
    res["ref_mean"] = float(np.mean([r for _, r in pairs]))
    res.update(summarize(pairs))
    res["within_1pt"] = bool(-1.0 <= res["ci95_pt"][0] and res["ci95_pt"][1] <= 1.0)
    res["wall_s"] = round(time.perf_counter() - t_start, 1)
    print(json.dumps({k: v for k, v in res.items() if k != "runs"}), flush=True)
    if args.out:
        with open(args.out, "w") as fo:
            json.dump(res, fo, indent=1)


def _collect(jobs, q, procs, ref, t_start, hip, args):
    import queue as _queue
    for i in range(len(jobs)):
        waited = 0
        while True:                           # a heartbeat line a minute: a silent run reads as hung
            try:
                msg = q.get(timeout=60)
                if msg[0] == "info":             # a worker's start record, not a result
                    args.worker_info[msg[1]] = msg[2]
                    print(f"  worker {msg[1]}: {msg[2]}", flush=True)
                    continue
                seed, u, acc, secs, mapped = msg
                if mapped:
                    args.worker_lib_mapped = True
                break
            except _queue.Empty:
                waited += 60
                print(f"  waiting for reference unit {i + 1}/{len(jobs)} "
                      f"({time.perf_counter() - t_start:.0f} s)", flush=True)
                if waited >= 3000 or not any(p.is_alive() for p in procs):
                    raise RuntimeError("reference workers stopped without a result")
        ref[(seed, u)] = acc
        print(f"  reference unit seed {seed} #{u}: {acc!r}% in {secs:.1f} s", flush=True)
        if i % 8 == 7 or i == len(jobs) - 1:
            print(f"  reference {i + 1}/{len(jobs)} units ({time.perf_counter() - t_start:.0f} s, "
                  f"last {secs:.1f} s)", flush=True)
            if args.out:                      # progress record: what a run cut off by its time limit had
                with open(args.out + ".partial", "w") as fo:
                    json.dump({"hip": {str(k): v for k, v in hip.items()},
                               "ref": [[sd, uu, a] for (sd, uu), a in ref.items()],
                               "elapsed_s": round(time.perf_counter() - t_start, 1)}, fo)
    for p in procs:
        p.join(timeout=120)


if __name__ == "__main__":
    main()
