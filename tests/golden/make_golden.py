"""Generate the golden vectors from the REFERENCE implementation (survey container only).

Run here, where /root/reference/src imports (torch CPU); never on the GPU box and never from a test:
    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden.py

It imports ``eegnet_repl.model.EEGNet`` from /root/reference/src/eegnet_repl/model.py:12-99 and runs
the reference hot loop (model.py:141-148 with train.py:94-103's Adam/CE) on seeded inputs.  Dropout
masks are injected through forward hooks on the two ``nn.Dropout`` modules (model.py:50,74) so the
outputs are reproducible; the masks are stored with the outputs.  Inputs x / labels are regenerated
from numpy PCG64 seeds by ``tests/golden/inputs.py`` and are not stored.

Fixture ids follow SURVEY.md section 8(c): G1..G7.
"""

from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, "/root/reference/src")

from inputs import make_inputs, make_masks  # noqa: E402
from eegnet_repl.model import EEGNet  # noqa: E402  (the reference)

import logging  # noqa: E402
logging.getLogger().setLevel(logging.WARNING)

torch.set_num_threads(8)


def sd_numpy(model):
    return {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def install_masks(model, p, masks):
    """Replace nn.Dropout's random draw with the given keep-masks (1 = keep)."""
    drops = [m for m in model.modules() if isinstance(m, nn.Dropout)]
    assert len(drops) == 2
    handles = []
    for mod, mk in zip(drops, masks):
        def hook(module, inp, out, mk=mk):
            if not module.training or p == 0.0:
                return out
            m = torch.as_tensor(mk, dtype=torch.float32).reshape(out.shape)
            return inp[0] * (m / (1.0 - p))
        handles.append(mod.register_forward_hook(hook))
    return handles


def run_case(name, C, T, B, F1=8, D=2, p=0.0, seed=0, steps=1, loss_scale=1.0, eval_case=False):
    torch.manual_seed(1000 + seed)
    model = EEGNet(C=C, T=T, F1=F1, D=D, p=p)
    if eval_case:
        # non-trivial running statistics (G3)
        g = torch.Generator().manual_seed(77 + seed)
        with torch.no_grad():
            for mod in model.modules():
                if isinstance(mod, nn.BatchNorm2d):
                    mod.running_mean.copy_(torch.randn(mod.num_features, generator=g) * 0.3)
                    mod.running_var.copy_(torch.rand(mod.num_features, generator=g) + 0.5)
                    mod.weight.copy_(torch.rand(mod.num_features, generator=g) + 0.5)
                    mod.bias.copy_(torch.randn(mod.num_features, generator=g) * 0.1)
    init = sd_numpy(model)
    x, y = make_inputs(B, C, T, seed)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    out = {"init." + k: v for k, v in init.items()}
    meta = dict(name=name, C=C, T=T, B=B, F1=F1, D=D, p=p, seed=seed, steps=steps,
                loss_scale=loss_scale, eval_case=eval_case, torch=torch.__version__,
                reference="PraKesEy/EEGNetReplication src/eegnet_repl/model.py")
    if eval_case:
        model.eval()
        with torch.no_grad():
            out["eval_logits"] = model(xt).numpy()
        out["meta"] = np.array(json.dumps(meta))
        return out
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, eps=1e-7, foreach=None, fused=None)
    loss_fn = nn.CrossEntropyLoss()
    losses = []
    model.train()
    for s in range(steps):
        masks = make_masks(B, F1 * D, T, seed * 100 + s, p) if p > 0 else (None, None)
        hs = install_masks(model, p, masks) if p > 0 else []
        logits = model(xt)
        loss = loss_fn(logits, yt)
        opt.zero_grad()
        (loss * loss_scale).backward()
        if s == 0:
            out["logits"] = logits.detach().numpy()
            out["loss"] = np.array(loss.item())
            for k, prm in model.named_parameters():
                out["grad." + k] = prm.grad.detach().numpy().copy()
            for k, v in sd_numpy(model).items():
                if "running" in k or "num_batches" in k:
                    out["buf1." + k] = v
            if p > 0:
                out["mask2"], out["mask3"] = masks
        opt.step()
        losses.append(loss.item())
        for hd in hs:
            hd.remove()
        if s == 0:
            for k, v in sd_numpy(model).items():
                out["step1." + k] = v
    out["losses"] = np.array(losses)
    for k, v in sd_numpy(model).items():
        out[f"final." + k] = v
    out["meta"] = np.array(json.dumps(meta))
    return out


CASES = [
    # EEGNet-8,2, 22x256, B=16, p=0, 3 Adam steps on the same batch
    dict(name="G1", C=22, T=256, B=16, p=0.0, seed=1, steps=3),
    # G2: same with p=0.5 and injected masks
    dict(name="G2", C=22, T=256, B=16, p=0.5, seed=2, steps=2),
    # G3: eval logits with non-trivial running stats
    dict(name="G3", C=22, T=256, B=16, p=0.5, seed=3, eval_case=True),
    # G4: real-data length T=257 (pool truncation)
    dict(name="G4", C=22, T=257, B=8, p=0.5, seed=4, steps=1),
    # G5: the reference test shapes (tests/test_model.py:110-114, 74, 42) and EEGNet-16,4 @ 64x512
    dict(name="G5_64x128", C=64, T=128, B=4, p=0.25, seed=51, steps=1),
    dict(name="G5_32x512", C=32, T=512, B=4, p=0.25, seed=52, steps=1),
    dict(name="G5_8x64", C=8, T=64, B=4, p=0.25, seed=53, steps=1),
    dict(name="G5_B1", C=22, T=256, B=1, p=0.0, seed=54, steps=1),
    dict(name="G5_F16D4", C=22, T=256, B=4, F1=16, D=4, p=0.25, seed=55, steps=1),
    dict(name="G5_16x4_64x512", C=64, T=512, B=4, F1=16, D=4, p=0.25, seed=56, steps=1),
    # G6: clamp-active (loss scaled by 1e3: spatial grads saturate at +-1, classifier at +-0.25)
    dict(name="G6", C=22, T=256, B=16, p=0.0, seed=6, steps=1, loss_scale=1000.0),
    # G7: 20-step Adam trajectory, p=0
    dict(name="G7", C=22, T=256, B=32, p=0.0, seed=7, steps=20),
]


def main():
    for case in CASES:
        out = run_case(**case)
        path = os.path.join(HERE, f"{case['name']}.npz")
        np.savez_compressed(path, **out)
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
