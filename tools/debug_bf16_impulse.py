"""Impulse probes of the bf16 eval kernel's spatial phase (traced build): x = e_(c0,t0) for a few
(c0, t0); prints where s[o, t] is non-zero against the expected s[:, t0] = ws[:, c0]."""
import ctypes
import os
import sys

import numpy as np
import torch

os.environ.setdefault("EEGNET_LIB", "libeegnet_hip_trace.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, _lib  # noqa: E402

C, T, F1, D = 64, 512, 16, 4
F2 = F1 * D
F2P, T1 = 64, T // 4
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = EEGNet(C, T, F1=F1, D=D).to(dev).eval()
ws = m.spatial.weight.detach().reshape(F2, C).cpu().numpy()
lib = _lib.load()
lib.eegnet_debug_bf16.argtypes = [ctypes.c_void_p]
buf = torch.zeros(F2P * (T + 2 * T1) + 64 * T, device=dev)
for c0, t0 in [(0, 0), (1, 0), (0, 1), (0, 5), (9, 37), (40, 300)]:
    x = torch.zeros(1, C, T, device=dev)
    x[0, c0, t0] = 1.0
    buf.zero_()
    lib.eegnet_debug_bf16(ctypes.c_void_p(buf.data_ptr()))
    with torch.no_grad():
        m(x.to(torch.bfloat16))
    torch.cuda.synchronize()
    lib.eegnet_debug_bf16(None)
    S = buf[:F2P * T].reshape(F2P, T).cpu().numpy()
    X = buf[F2P * (T + 2 * T1):].reshape(64, T).cpu().numpy()
    print("   x image nonzeros:", np.argwhere(X != 0).tolist()[:6], "values", X[X != 0][:6])
    nz = np.argwhere(S != 0)
    ts = sorted(set(nz[:, 1].tolist()))
    print(f"impulse c={c0} t={t0}: nonzero t columns {ts[:10]} count {len(nz)}")
    for t in ts[:3]:
        col = S[:, t]
        # which ws column does it match?
        best = np.abs(ws.T - col[None, :F2]).sum(1)
        print(f"   t={t}: s[:4,t]={col[:4]} best-matching ws column c={best.argmin()} (err {best.min():.3e}); ws[:4,c0]={ws[:4, c0]}")
        rows = np.argwhere(col != 0).ravel()
        print(f"   nonzero rows {rows[:16].tolist()} ... ({len(rows)})")
