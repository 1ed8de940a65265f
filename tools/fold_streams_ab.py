"""A rank's fold share as one fold batch (one launch per pass for all its folds) or as G fold batches
on G streams (the same per-fold kernels and numerics: a fold's launch geometry depends on its own
B = 64 only), so that one batch's reduction / finalize tails overlap another's loops."""
import os, sys, time, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, FoldBatch

dev = torch.device("cuda:0")
rng = np.random.default_rng(77)
X = torch.from_numpy(rng.standard_normal((1440, 22, 257), dtype=np.float32)).to(dev)
y = torch.from_numpy(rng.integers(0, 4, 1440)).to(dev)
EP = 8
out = {}


def run(k, groups, graphs=True):
    torch.manual_seed(3)
    models = [EEGNet(22, 257, p=0.5).to(dev).train() for _ in range(k)]
    gens = [torch.Generator().manual_seed(100 + j) for j in range(k)]
    cut = np.array_split(np.arange(k), groups)
    fbs = [FoldBatch([models[j] for j in c], [int(j) for j in c], graphs=graphs, fused=True) for c in cut]
    sts = [torch.cuda.Stream() for _ in cut]
    cur = torch.cuda.current_stream()

    def epoch():
        for fb, c, s in zip(fbs, cut, sts):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                fb.epoch([(X, y)] * len(c), 64, [gens[j] for j in c])
        for s in sts:
            cur.wait_stream(s)

    epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(EP):
        epoch()
    torch.cuda.synchronize()
    r = k * 1440 * EP / (time.perf_counter() - t0)
    losses = [float(models[j].training) for j in range(1)]
    return r


GRAPHS = os.environ.get("GRAPHS", "1") == "1"
SWEEP = json.loads(os.environ.get("SWEEP", "[[12, [1, 2, 3]], [90, [1, 2]]]"))
for rep in range(int(os.environ.get("REPS", "3"))):
    for k, gs in SWEEP:
        for g in gs:
            r = run(k, g, GRAPHS)
            out.setdefault(f"{k} folds x {g} streams graphs={GRAPHS}", []).append(round(r / 1e6, 3))
            print(k, g, round(r / 1e6, 3), flush=True)
print(json.dumps(out))
