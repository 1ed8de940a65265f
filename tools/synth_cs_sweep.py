"""Learnability of synthetic-session presets: the HIP protocols at the reference's
500 epochs on sessions drawn with each preset's population / subject parameters -- cross-subject
(train.py:151-291: 90 folds, p = 0.25, batch 64, final weights) and, with --ws, within-subject
(train.py:30-148: 36 units, p = 0.5) -- printing the mean test accuracy and the per-test-subject means.
A preset is (mu band, beta band, class-effect strength, spatial-mixing jitter); "v1" is round 3's
generator.  The accuracy-parity specs (tools/accuracy_parity.py) are reused, so a preset's numbers are
what that tool's HIP side reports.

    python tools/synth_cs_sweep.py v1 v2 ...  [--epochs 500] [--ws]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from eegnetreplication_amd import dataset as D  # noqa: E402

PRESETS = {
    "v1": dict(mu=(9.0, 11.5), beta=(19.0, 24.0), strength=(0.25, 0.6), mix=0.15),
    "v2": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.3, 0.6), mix=0.10),
    "v3": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.25, 0.5), mix=0.10),
    "v4": dict(mu=(9.2, 10.8), beta=(19.5, 22.5), strength=(0.3, 0.6), mix=0.12),
    "v5": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.4, 0.7), mix=0.05),
    "v6": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.35, 0.65), mix=0.08),
    "v7": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.3, 0.6), mix=0.06),
    "v8": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.4, 0.7), mix=0.08),
    "v9": dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.35, 0.65), mix=0.06),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("presets", nargs="+")
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--ws", action="store_true", help="also the within-subject protocol")
    args = ap.parse_args()
    from eegnetreplication_amd.train import _run_units
    from accuracy_parity import cs_specs, ws_specs
    dev = torch.device("cuda:0")
    for name in args.presets:
        D.SYNTH_PARAMS.update(PRESETS[name])
        for proto in (("cs", "ws") if args.ws else ("cs",)):
            specs = cs_specs(0, list(range(90))) if proto == "cs" else ws_specs(0)
            t0 = time.perf_counter()
            out = _run_units(specs, args.epochs, dev, len(specs))
            acc = np.array([r["test_acc"] for r in out])
            per_s = 10 if proto == "cs" else 4
            per = [float(acc[per_s * s:per_s * s + per_s].mean()) for s in range(9)]
            print(f"{name} {PRESETS[name]}: {proto} {acc.mean():.2f}% (per subject "
                  f"{' '.join(f'{a:.1f}' for a in per)}), {time.perf_counter() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
