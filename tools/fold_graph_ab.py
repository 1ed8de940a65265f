"""Fold-indexed epochs at a rank share with and without the epoch hipGraph (FoldBatch graphs=True /
False, fused=True), alternating: do the graph's kernel nodes cost the fold step anything?"""
import os, sys, time, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, FoldBatch

dev = torch.device("cuda:0")
rng = np.random.default_rng(77)
X = torch.from_numpy(rng.standard_normal((1440, 22, 257), dtype=np.float32)).to(dev)
y = torch.from_numpy(rng.integers(0, 4, 1440)).to(dev)
out = {}
for rep in range(2):
    for k in (12, 90):
        for graphs in (True, False):
            torch.manual_seed(3)
            fb = FoldBatch([EEGNet(22, 257, p=0.5).to(dev).train() for _ in range(k)], list(range(k)),
                           graphs=graphs, fused=True)
            gens = [torch.Generator().manual_seed(100 + j) for j in range(k)]
            fb.epoch([(X, y)] * k, 64, gens)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(8):
                fb.epoch([(X, y)] * k, 64, gens)
            torch.cuda.synchronize()
            r = k * 1440 * 8 / (time.perf_counter() - t0)
            out.setdefault(f"{k} graphs={graphs}", []).append(round(r / 1e6, 3))
            del fb
            print(k, graphs, round(r / 1e6, 3), flush=True)
print(json.dumps(out))
