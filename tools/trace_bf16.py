"""Phase breakdown of the cfg5 bf16 eval kernel (traced build, k_infer_bf16_cfg5): thread 0's shader
cycles per phase, summed over its workgroup's trials, averaged over the workgroups.
Phases: 0 wait for the chunk's x DMA (+ barrier) | 1 spatial GEMM | 2 barrier after it | 3 FIR + ELU +
pool4 | 4 the tail's barriers | 5 depthwise | 6 pointwise + classifier | 7 logits + next DMA issue."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

os.environ.setdefault("EEGNET_LIB", "libeegnet_hip_trace.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = EEGNet(64, 512, F1=16, D=4).to(dev).eval()
x = torch.randn(B, 64, 512, device=dev).to(torch.bfloat16)
lib = _lib.load()
lib.eegnet_debug_bf16.argtypes = [ctypes.c_void_p]
with torch.no_grad():
    m(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        m(x)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    buf = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    lib.eegnet_debug_bf16(ctypes.c_void_p(buf.data_ptr()))
    m(x)
    torch.cuda.synchronize()
    lib.eegnet_debug_bf16(None)
ph = buf.view(-1, 8).cpu().numpy()
ph = ph[ph.sum(1) > 0]
names = ["dma wait", "spatial", "barrier1", "fir+elu", "tail barriers", "depthwise", "pointwise", "logits+dma"]
tot = ph.sum(1).mean()
print(f"B={B}: {dt * 1e6:.1f} us per launch ({B / dt / 1e6:.2f} M trials/s), {len(ph)} workgroups, "
      f"{tot / max(1, B / len(ph)):.0f} cycles per trial per workgroup")
for k, n in enumerate(names):
    print(f"  {n:14s} {ph[:, k].mean() / (B / len(ph)):9.0f} cycles/trial  {100 * ph[:, k].mean() / tot:5.1f} %")
