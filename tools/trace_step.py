"""Timeline of one EEGNet train step from the kernels' own stamps (eegnet_trace_enable).

    python tools/trace_step.py [--batch B]

Per pass: launch skew, prologue, trial loop, publish, group/top reduction, finalize (µs, wall clock
at 100 MHz), the gap to the next kernel, and the shader-clock in-loop phase sums per trial.
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

NAMES = ["A", "B", "C", "D", "E", "infer"]
SLOTS, MAXWG = 16, 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--C", type=int, default=22)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--F1", type=int, default=8)
    ap.add_argument("--D", type=int, default=2)
    ap.add_argument("--dump", default=None, help="save the raw stamp array (.npy)")
    args = ap.parse_args()
    from eegnetreplication_amd import EEGNet, FusedTrainer, _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = EEGNet(args.C, args.T, F1=args.F1, D=args.D, p=0.5).to(dev).train()
    rng = np.random.default_rng(1234)
    x = torch.from_numpy(rng.standard_normal((args.batch, args.C, args.T), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.integers(0, 4, args.batch)).to(dev)
    tr = FusedTrainer(model)
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
    grids = [int((a[p, :, 0] > 0).sum()) for p in range(5)]
    grid = grids[0]
    t0 = min(a[p, :grids[p], 0].min() for p in range(5) if grids[p])
    us = lambda v: (v - t0) / 100.0   # 100 MHz wall clock -> µs from pass A's first entry
    prev_end = None
    ntr = max(1, args.batch // grid)
    print(f"grids {grids} workgroups")
    for p in range(5):
        if not grids[p]:                      # (the wide step stamps passes A and E only)
            continue
        st = a[p, :grids[p]]
        F2 = args.F1 * args.D                 # the wide streaming passes: NOC o-chunk workgroups per trial
        noc = (F2 + 15) // 16 if F2 > 16 else 1
        ntr = max(1, args.batch * noc // grids[p])
        ent, pro, loop, pub = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
        grp = st[:, 4][st[:, 4] > 0]
        top = st[:, 5][st[:, 5] > 0]
        fin = st[:, 6][st[:, 6] > 0]
        end = max(v.max() for v in (pub, grp, top, fin) if len(v))
        line = (f"pass {NAMES[p]}: start {us(ent.min()):7.1f} (skew {(ent.max()-ent.min())/100:5.1f})"
                f" | prologue {np.mean(pro-ent)/100:5.1f} | loop avg {np.mean(loop-pro)/100:6.1f} max {np.max(loop-pro)/100:6.1f}"
                f" | publish {np.mean(pub-loop)/100:5.1f} | last pub {us(pub.max()):7.1f}")
        if len(grp):
            line += f" | grp-red {(grp.max()-pub.max())/100:5.1f}"
        if len(top):
            line += f" | top {(top.max()-(grp.max() if len(grp) else pub.max()))/100:5.1f}"
        if len(fin):
            line += f" | fin {(fin.max()-top.max())/100:5.1f}"
        line += f" | end {us(end):7.1f}"
        if prev_end is not None:
            line += f" | gap {(ent.min()-prev_end)/100:5.1f}"
        prev_end = end
        print(line)
        fs = a[6, p]
        if fs[3] > 0:
            ks = [k for k in range(16) if fs[k] > 0]
            print("    reduce/finalize stamps (µs after last publish):",
                  " ".join(f"{k}:{(fs[k]-pub.max())/100:.2f}" for k in ks))
        if p == 4:
            ps = a[7, :grids[p], :8]
            ks = [k for k in range(8) if (ps[:, k] > 0).any()]
            if ks:
                print("    prologue stamps (µs after entry, mean over workgroups):",
                      " ".join(f"{k}:{np.mean(ps[:, k]-ent)/100:.2f}" for k in ks), f"pro:{np.mean(pro-ent)/100:.2f}")
        if p == 2:
            ps = a[7, :grids[p], 8:12]
            if (ps > 0).any():
                print("    tail stamps (µs after the loop, mean over workgroups): "
                      "waves joined %.2f | sdz reduced %.2f | rows in LDS %.2f | row published %.2f"
                      % tuple(np.mean(ps[:, k] - loop) / 100 for k in range(4)))
        if os.environ.get("SLOWEST"):
            # the workgroups whose loops end last: index, XCD (index mod 8), entry, prologue and loop (µs)
            le = loop - t0
            idx = np.argsort(-le)[:8]
            print("    last loop ends:", " ".join(f"wg{i}(x{i % 8}) e{(ent[i]-t0)/100:.1f} p{(pro[i]-ent[i])/100:.1f} l{(loop[i]-pro[i])/100:.1f}" for i in idx))
            bx = [np.mean((loop - pro)[np.arange(len(loop)) % 8 == x]) / 100 for x in range(8)]
            print("    loop avg by XCD:", " ".join(f"{v:.1f}" for v in bx), "| wg0 loop", f"{(loop[0]-pro[0])/100:.1f}", "prologue", f"{(pro[0]-ent[0])/100:.1f}")
        ph = st[:, 8:16].mean(axis=0) / ntr
        if ph.any():
            print("    in-loop phases (shader cycles per trial, wave 0):", " ".join(f"{v:.0f}" for v in ph))


if __name__ == "__main__":
    main()
