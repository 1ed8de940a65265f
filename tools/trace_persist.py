"""Timeline of one persistent train step (k_step, csrc/eegnet_persist.hip) from its own stamps.

    python tools/trace_persist.py [--batch B] [--T 256]

Per phase (µs from the kernel's first workgroup entry, 100 MHz wall clock; mean / max over the
workgroups): the phase's start (its body entered: the previous reduction's hook is inside the body's
prologue), the loop start, the loop end, the partial row published; then the phase's grid reduction:
first barrier passed, column totals in LDS (second barrier), the finalize done.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("EEGNET_LIB", "libeegnet_hip_trace.so")
sys.path.insert(0, ROOT)

SLOTS, MAXWG = 16, 2048
NAMES = "ABCDE"
EV = {"entry": 0, "pro": 1, "loop": 2, "pub": 3, "bar1": 4, "totals": 5, "fin": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--dump", default=None)
    args = ap.parse_args()
    from eegnetreplication_amd import EEGNet, FusedTrainer, _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = EEGNet(22, args.T, p=0.5).to(dev).train()
    rng = np.random.default_rng(1234)
    x = torch.from_numpy(rng.standard_normal((args.batch, 22, args.T), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.integers(0, 4, args.batch)).to(dev)
    tr = FusedTrainer(model, persist=True)
    for _ in range(5):
        tr.step(x, y)
    nb = lib.eegnet_trace_bytes()
    buf = torch.zeros(nb // 8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    lib.eegnet_trace_enable(ctypes.c_void_p(buf.data_ptr()))
    tr.step(x, y)
    torch.cuda.synchronize()
    lib.eegnet_trace_enable(None)
    a = buf.cpu().numpy().reshape(8, MAXWG, SLOTS).astype(np.float64)
    if args.dump:
        np.save(args.dump, a)
    G = int((a[0, :, 0] > 0).sum())
    st = a[:5, :G]
    t0 = st[0, :, 0].min()
    us = lambda v: (v - t0) / 100.0
    print(f"k_step: {G} workgroups, B = {args.batch}, T = {args.T}")
    print(f"{'phase':5s} {'start':>13s} {'loop start':>13s} {'loop end':>13s} {'published':>13s} | "
          f"{'barrier 1':>13s} {'totals':>13s} {'finalized':>13s}   (mean / max)")
    for p in range(5):
        cells = []
        for ev in ("entry", "pro", "loop", "pub", "bar1", "totals", "fin"):
            v = st[p, :, EV[ev]]
            v = v[v > 0]
            cells.append(f"{us(v).mean():6.1f}/{us(v).max():6.1f}" if len(v) else f"{'-':>13s}")
        print(f"{NAMES[p]:5s} " + " ".join(cells[:4]) + " | " + " ".join(cells[4:]))
    end = st[4, :, EV["fin"]]
    print(f"step (first entry -> last finalize): {us(end[end > 0]).max():.1f} us")


if __name__ == "__main__":
    main()
