"""Real-protocol fold-launch throughput at a given EEGNET_FOLD_TPW (read once per process): the
fused fold-indexed leg of bench.py's bench_folds only, at several fold-batch widths.
    EEGNET_LIB=libeegnet_hip_t28.so python tools/fold_tpw_sweep.py 90 12   (a -DEEGNET_FOLD_TPW_S / _C build)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, FoldBatch  # noqa: E402


def run(n_folds, n_train=1440, epochs=2, dev="cuda:0"):
    C, T = 22, 257
    rng = np.random.default_rng(77)
    X = torch.from_numpy(rng.standard_normal((n_train, C, T), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.integers(0, 4, n_train)).to(dev)
    torch.manual_seed(3)
    models = [EEGNet(C, T, p=0.5).to(dev).train() for _ in range(n_folds)]
    fb = FoldBatch(models, list(range(n_folds)), graphs=True, fused=True)
    gens = [torch.Generator().manual_seed(100 + k) for k in range(n_folds)]
    fb.epoch([(X, y)] * n_folds, 64, gens)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(epochs):
        fb.epoch([(X, y)] * n_folds, 64, gens)
    torch.cuda.synchronize()
    return n_folds * n_train * epochs / (time.perf_counter() - t0)


if __name__ == "__main__":
    tpw = os.environ.get("EEGNET_LIB", "libeegnet_hip.so")
    for nf in [int(a) for a in sys.argv[1:]] or [90, 12]:
        print(f"tpw {tpw} folds {nf}: {run(nf, epochs=int(os.environ.get('EPOCHS', 2))) / 1e6:.3f} M trials/s",
              flush=True)
