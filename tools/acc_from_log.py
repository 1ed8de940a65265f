"""Rebuild an accuracy_parity.py result from a run cut off by its time limit before the tool could
write it (round 4's chunk acc_cs_common_b): the HIP accuracies from the .partial progress record, the
reference accuracies from the per-unit log lines (printed to 2 decimals there; a test accuracy is
k / n_test, so the exact value is recovered as round(acc * n_test / 100) / n_test).

    python tools/acc_from_log.py LOG PARTIAL OUT.json --protocol cs --dropout common --epochs 500 \\
        --folds 20 ... 35 --seeds 0 1 2 [--n-test 288]
"""
import argparse
import json
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from accuracy_parity import summarize  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("partial")
    ap.add_argument("out")
    ap.add_argument("--protocol", default="cs")
    ap.add_argument("--dropout", default="common")
    ap.add_argument("--epochs", type=int, default=500)
    ap.add_argument("--folds", type=int, nargs="+", required=True)
    ap.add_argument("--seeds", type=int, nargs="+", required=True)
    ap.add_argument("--n-test", type=int, default=288)
    args = ap.parse_args()
    part = json.load(open(args.partial))
    ref = {}
    for line in open(args.log):
        m = re.match(r"  reference unit seed (\d+) #(\d+): ([\d.]+)% in", line)
        if m:
            k = round(float(m.group(3)) * args.n_test / 100.0)
            ref[(int(m.group(1)), int(m.group(2)))] = 100.0 * k / args.n_test
    res = {"protocol": f"cross-subject (train.py:151-291), p = 0.25, folds {args.folds}" if args.protocol == "cs"
           else "within-subject (train.py:30-148), p = 0.5",
           "data": "seeded synthetic SMR sessions (dataset.synthetic_session); rebuilt from the run log",
           "epochs": args.epochs, "seeds": args.seeds, "dropout": args.dropout, "runs": [], "complete": False}
    pairs = []
    for sd in args.seeds:
        hip = part["hip"][str(sd)]
        us = [u for u in range(len(hip)) if (sd, u) in ref]
        h = [hip[u] for u in us]
        r = [ref[(sd, u)] for u in us]
        res["runs"].append({"seed": sd, "units": us, "hip": h, "ref": r, "hip_mean": float(np.mean(h)),
                            "ref_mean": float(np.mean(r)), "diff_pt": float(np.mean(h) - np.mean(r))})
        pairs += list(zip(h, r))
    res["missing"] = [[sd, args.folds[u]] for sd in args.seeds for u in range(len(part["hip"][str(sd)]))
                      if (sd, u) not in ref]
    res["hip_mean"] = float(np.mean([h for h, _ in pairs]))
    res["ref_mean"] = float(np.mean([r for _, r in pairs]))
    res.update(summarize(pairs))
    res["within_1pt"] = bool(-1.0 <= res["ci95_pt"][0] and res["ci95_pt"][1] <= 1.0)
    with open(args.out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "runs"}))


if __name__ == "__main__":
    main()
