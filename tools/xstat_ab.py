"""What the per-trial BN1 x-statistics table saves pass A at a large batch: one fold, batch B, fused
fold-indexed launches, with (xstats=True) and without the table, alternating; per-kernel average
µs from the library's HIP-event profile.

    python tools/xstat_ab.py [--batch 4096] [--C 22] [--T 256] [--epochs 6] [--rounds 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--C", type=int, default=22)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    from eegnetreplication_amd import EEGNet, _lib
    from eegnetreplication_amd.folds import FoldBatch
    dev = torch.device("cuda", 0)
    n = 4 * args.batch
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn(n, args.C, args.T, device=dev, generator=g)
    y = torch.randint(0, 4, (n,), device=dev, generator=g)
    for r in range(args.rounds):
        for xs in (False, True):
            torch.manual_seed(0)
            m = EEGNet(args.C, args.T, p=0.5).to(dev).train()
            fb = FoldBatch([m], [0], fused=True, xstats=xs)
            gens = [torch.Generator().manual_seed(5)]
            for _ in range(2):
                fb.epoch([(X, y)], batch_size=args.batch, generators=gens)
            torch.cuda.synchronize()
            _lib.profile_enable(True)
            for _ in range(args.epochs):
                fb.epoch([(X, y)], batch_size=args.batch, generators=gens)
            torch.cuda.synchronize()
            kern = _lib.profile_collect()
            _lib.profile_enable(False)
            tot = sum(t for _, t in kern.values()) / (4 * args.epochs)
            print(f"round {r} xstats={int(xs)}: {tot * 1e3:.1f} us/step of kernels; "
                  + ", ".join(f"{k} {t / max(c, 1) * 1e3:.1f}" for k, (c, t) in sorted(kern.items())), flush=True)
    # the table itself: one batch of B trials through eegnet_x_stats
    from eegnetreplication_amd import ops
    shape = m.shape
    xb = X[:args.batch]
    out = ops.x_stats(shape, xb)
    for _ in range(3):
        ops.x_stats(shape, xb, out=out)
    torch.cuda.synchronize()
    _lib.profile_enable(True)
    for _ in range(20):
        ops.x_stats(shape, xb, out=out)
    torch.cuda.synchronize()
    kern = _lib.profile_collect()
    _lib.profile_enable(False)
    print("x_stats of one batch: " + ", ".join(f"{k} {t / max(c, 1) * 1e3:.1f} us" for k, (c, t) in kern.items()),
          flush=True)


if __name__ == "__main__":
    main()
