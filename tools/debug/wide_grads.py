"""Debug: per-tensor errors of the wide train step against the float64 oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(sys.path[0], "tests"))
import numpy as np, torch
from golden_util import make_inputs, make_masks
from hip_cases import random_model, oracle_step, grads_of

for (C, T, F1, D, B, p) in [(64, 512, 16, 4, 24, 0.25), (22, 256, 12, 2, 16, 0.0), (22, 256, 8, 2, 16, 0.0)]:
    m = random_model(C, T, F1=F1, D=D, p=p, seed=1)
    x_np, y_np = make_inputs(B, C, T, 5)
    masks = make_masks(B, F1 * D, T, 6, p) if p > 0 else None
    rl, rloss, rg, rnb, _ = oracle_step(m, x_np, y_np, p=p, masks=masks)
    m = m.cuda().train()
    if masks is not None:
        m.set_dropout_masks(torch.from_numpy(masks[0]).cuda(), torch.from_numpy(masks[1]).cuda())
    lg = m(torch.from_numpy(x_np).cuda())
    torch.nn.functional.cross_entropy(lg, torch.from_numpy(y_np).cuda()).backward()
    g = grads_of(m)
    print(f"== EEGNet-{F1},{D} {C}x{T} B={B}")
    for k in rg:
        e = np.abs(g[k] - rg[k]).max() / max(np.abs(rg[k]).max(), 1e-30)
        print(f"  {k:24s} rel {e:.3e}  scale {np.abs(rg[k]).max():.3e}")
    bufs = {k: b.detach().cpu().numpy() for k, b in m.named_buffers()}
    for k, v in rnb.items():
        v = np.asarray(v, np.float64)
        print(f"  {k:36s} absdiff {np.abs(bufs[k] - v).max():.3e} scale {np.abs(v).max():.3e}")
