"""Where the constant of the bench's timed region goes (driver flags: 20 steps): wall time of K fused
cfg2 steps for several K in one process (fit t = c + K s), and the host-side cost of one
trainer.step call (enqueue only, the GPU busy behind it)."""
import sys, os, time, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, FusedTrainer

dev = torch.device("cuda:0")
B, C, T = 4096, 22, 256
torch.manual_seed(0)
model = EEGNet(C, T, F1=8, D=2, p=0.5).to(dev).train()
xs = [torch.randn(B, C, T, device=dev) for _ in range(4)]
ys = [torch.randint(0, 4, (B,), device=dev) for _ in range(4)]
tr = FusedTrainer(model)
for i in range(30):
    tr.step(xs[i % 4], ys[i % 4])
torch.cuda.synchronize()
res = {}
for rep in range(3):
    for K in (5, 10, 20, 40, 80):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            tr.step(xs[i % 4], ys[i % 4])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res.setdefault(K, []).append((t2 - t0, t1 - t0))
Ks = sorted(res)
tot = [min(r[0] for r in res[k]) for k in Ks]
enq = [min(r[1] for r in res[k]) for k in Ks]
s, c = np.polyfit(Ks, tot, 1)
se, ce = np.polyfit(Ks, enq, 1)
print(json.dumps({"K": Ks, "wall_ms": [round(1e3 * v, 4) for v in tot], "enqueue_ms": [round(1e3 * v, 4) for v in enq],
                  "fit_step_us": round(1e6 * s, 2), "fit_const_us": round(1e6 * c, 1),
                  "enqueue_per_step_us": round(1e6 * se, 2), "enqueue_const_us": round(1e6 * ce, 1)}))
