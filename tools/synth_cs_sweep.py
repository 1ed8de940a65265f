"""Cross-subject learnability of synthetic-session presets: the HIP cross-subject
protocol (train.py:151-291: 90 folds, p = 0.25, batch 64, final weights) at the reference's 500 epochs
on sessions drawn with each preset's population / subject parameters; prints the mean test accuracy
over the 90 folds and per test subject.  A preset is (mu band, beta band, class-effect strength,
spatial-mixing jitter); "v1" is round 3's generator.

    python tools/synth_cs_sweep.py v1 v2 ...  [--epochs 500]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import dataset as D  # noqa: E402

PRESETS = {
    "v1": dict(mu=(9.0, 11.5), beta=(19.0, 24.0), strength=(0.25, 0.6), mix=0.15),
    "v2": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.3, 0.6), mix=0.10),
    "v3": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.25, 0.5), mix=0.10),
    "v4": dict(mu=(9.2, 10.8), beta=(19.5, 22.5), strength=(0.3, 0.6), mix=0.12),
    "v5": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.4, 0.7), mix=0.05),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("presets", nargs="+")
    ap.add_argument("--epochs", type=int, default=500)
    args = ap.parse_args()
    from eegnetreplication_amd.train import _run_units, cross_subject_units
    dev = torch.device("cuda:0")
    units = cross_subject_units()
    for name in args.presets:
        D.SYNTH_PARAMS.update(PRESETS[name])
        sess = {}

        def get(s, mode):
            if (s, mode) not in sess:
                sess[(s, mode)] = D.synthetic_session(s, mode)
            return sess[(s, mode)]
        specs = []
        for u, (s, k, trs, vas) in enumerate(units):
            X = np.concatenate([get(v, "Train").X for v in trs + vas])
            y = np.concatenate([get(v, "Train").y for v in trs + vas])
            ntr = sum(len(get(v, "Train").y) for v in trs)
            ids = np.arange(len(y))
            te = get(s, "Eval")
            specs.append((X, y, ids[:ntr], ids[ntr:], (te.X, te.y), 0.25, u))
        t0 = time.perf_counter()
        out = _run_units(specs, args.epochs, dev, len(specs))
        acc = np.array([r["test_acc"] for r in out])
        per = [float(acc[10 * s:10 * s + 10].mean()) for s in range(9)]
        print(f"{name} {PRESETS[name]}: cross-subject {acc.mean():.2f}% (per test subject "
              f"{' '.join(f'{a:.1f}' for a in per)}), {time.perf_counter() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
