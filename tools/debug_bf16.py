"""Phase-by-phase check of the bf16 eval kernel (traced build): dumps workgroup 0's first trial's
s, a, z planes and compares them with a float64 numpy restatement of the same phases."""
import ctypes
import os
import sys

import numpy as np
import torch

os.environ.setdefault("EEGNET_LIB", "libeegnet_hip_trace.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, _lib  # noqa: E402

C, T, F1, D = [int(a) for a in sys.argv[1:5]] if len(sys.argv) > 4 else (64, 512, 16, 4)
F2 = F1 * D
F2P = 16 if F2 <= 16 else 32 if F2 <= 32 else 64
T1 = T // 4
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = EEGNet(C, T, F1=F1, D=D).to(dev).eval()
with torch.no_grad():
    for n, b in m.named_buffers():
        if n.endswith("running_var"):
            b.uniform_(0.5, 1.5)
x = torch.randn(2, C, T, device=dev).to(torch.bfloat16)
lib = _lib.load()
lib.eegnet_debug_bf16.argtypes = [ctypes.c_void_p]
buf = torch.zeros(F2P * (T + 2 * T1) + 64 * T, device=dev)
lib.eegnet_debug_bf16(ctypes.c_void_p(buf.data_ptr()))
with torch.no_grad():
    out = m(x)
torch.cuda.synchronize()
lib.eegnet_debug_bf16(None)
d = buf.cpu().numpy().astype(np.float64)
S, A, Z = d[:F2P * T].reshape(F2P, T), d[F2P * T:F2P * (T + T1)].reshape(F2P, T1), d[F2P * (T + T1):F2P * (T + 2 * T1)].reshape(F2P, T1)

P = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.named_parameters()}
Bf = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.named_buffers()}
x0 = x[0].float().cpu().numpy().astype(np.float64)
ws = P["spatial.weight"].reshape(F2, C)
s = ws @ x0
w1 = P["temporal.0.weight"].reshape(F1, -1)
K1 = w1.shape[1]
Pp = (K1 - 1) // 2
sp = np.pad(s, ((0, 0), (Pp, K1 - 1 - Pp)))
v = np.stack([np.array([np.dot(w1[o // D], sp[o, t:t + K1]) for t in range(T)]) for o in range(F2)])
eps = 1e-5
a1 = P["temporal.1.weight"] / np.sqrt(Bf["temporal.1.running_var"] + eps)
c1 = P["temporal.1.bias"] - a1 * Bf["temporal.1.running_mean"]
s2 = P["aggregation.0.weight"] / np.sqrt(Bf["aggregation.0.running_var"] + eps)
g = np.arange(F2) // D
al = a1[g] * s2
be = (c1[g] * ws.sum(1) - Bf["aggregation.0.running_mean"]) * s2 + P["aggregation.0.bias"]
zz = al[:, None] * v + be[:, None]
e = np.where(zz > 0, zz, np.expm1(np.minimum(zz, 0)))
a = e[:, :4 * T1].reshape(F2, T1, 4).mean(-1)
w2 = P["block_2.0.weight"].reshape(F2, 16)
ap = np.pad(a, ((0, 0), (7, 8)))
z = np.stack([np.array([np.dot(w2[o], ap[o, t:t + 16]) for t in range(T1)]) for o in range(F2)])


def rep(name, got, ref):
    err = np.abs(got - ref)
    i = np.unravel_index(err.argmax(), err.shape)
    print(f"{name}: max|err| {err.max():.4e} at {i} (got {got[i]:.5f} ref {ref[i]:.5f}); max|ref| {np.abs(ref).max():.4e}")


rep("s", S[:F2], s)
rep("a", A[:F2], a)
rep("z", Z[:F2], z)
print("s[0,:8]", S[0, :8], "\nref", s[0, :8])
print("a[0,:8]", A[0, :8], "\nref", a[0, :8])
print("z[0,:8]", Z[0, :8], "\nref", z[0, :8])
print("logits", out.cpu().numpy())
