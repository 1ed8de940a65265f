"""Eager vs hipGraph-replayed fused train step at B=4096 (dropout keys from the device step)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, ops  # noqa: E402
from eegnetreplication_amd.model import FusedAdamState  # noqa: E402

dev = torch.device("cuda:0")
B, C, T = 4096, 22, 256
torch.manual_seed(0)
m = EEGNet(C, T, p=0.5).to(dev)
rng = np.random.default_rng(1234)
x = torch.from_numpy(rng.standard_normal((B, C, T), dtype=np.float32)).to(dev)
y = torch.from_numpy(rng.integers(0, 4, B)).to(dev)
a = FusedAdamState(m)
loss = torch.zeros(1, device=dev)
ws = ops.new_workspace(m.shape, B, dev)


def step():
    ops.train_step(m.shape, m.flat_parameters(), m.flat_bn_buffers(), x, y, 5, 0, a.grads, a.state,
                   a.step, ws, loss, nbt=m.flat_num_batches_tracked(), key_from_step=True)


for _ in range(10):
    step()
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    step()
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        step()
    torch.cuda.synchronize()
    te = (time.perf_counter() - t0) / 100
    t0 = time.perf_counter()
    for _ in range(100):
        g.replay()
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / 100
    print(f"eager {te * 1e6:.1f} us ({B / te / 1e6:.2f} M/s)  graph {tg * 1e6:.1f} us ({B / tg / 1e6:.2f} M/s)")
print("finite", bool(torch.isfinite(loss).all()))
