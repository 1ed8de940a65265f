"""Host enqueue cost of FusedTrainer.step vs device time (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from eegnetreplication_amd import EEGNet, FusedTrainer
dev = torch.device("cuda:0")
m = EEGNet(22, 256, p=0.5).to(dev).train()
x = torch.randn(4096, 22, 256, device=dev); y = torch.randint(0, 4, (4096,), device=dev)
tr = FusedTrainer(m)
for _ in range(10): tr.step(x, y)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(50): tr.step(x, y)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e6*(t1-t0)/50:.1f} us/step, total {1e6*(t2-t0)/50:.1f} us/step", flush=True)
xs = x[:64].contiguous(); ys = y[:64].contiguous()
for rep in range(2):
    t0 = time.perf_counter()
    for _ in range(200): tr.step(xs, ys)
    t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"B=64: enqueue {1e6*(t1-t0)/200:.1f} us/step, total {1e6*(t2-t0)/200:.1f} us/step", flush=True)
import cProfile, pstats
pr = cProfile.Profile(); pr.enable()
for _ in range(200): tr.step(xs, ys)
pr.disable(); torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(8)
