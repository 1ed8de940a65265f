"""Equivalence test (TOST) of the accuracy-parity records against the north_star's +-1 pt margin.

A 95 % confidence interval that must fit inside [-1, +1] pt is a stricter test than "equivalent within
1 pt": the two one-sided tests (Schuirmann's TOST) at alpha = 0.05 reject "the mean paired difference is
<= -1 pt" and "... >= +1 pt" each at 5 %, which is the same as the 90 % interval lying inside the margin.
Reads the merged records of tools/accuracy_parity.py / acc_merge.py (their `runs[].hip` / `runs[].ref`
per-unit accuracies) and recomputes the paired statistics from the units themselves.

    python tools/acc_tost.py profiles/r4_accuracy_cs_e500_s4_indep.json [...] [--margin 1.0] [--json OUT]
"""
import argparse
import json
import math
import sys

import numpy as np
from scipy import stats


def paired_diffs(rec):
    d = []
    for run in rec["runs"]:
        for h, r in zip(run["hip"], run["ref"]):
            d.append(float(h) - float(r))
    return np.asarray(d, dtype=np.float64)


def tost(d, margin):
    n = len(d)
    mean = float(d.mean())
    sd = float(d.std(ddof=1))
    se = sd / math.sqrt(n)
    df = n - 1
    t90 = float(stats.t.ppf(0.95, df))
    t95 = float(stats.t.ppf(0.975, df))
    # H0a: mu <= -margin  (reject for large t_lo);  H0b: mu >= +margin  (reject for small t_hi)
    t_lo = (mean + margin) / se
    t_hi = (mean - margin) / se
    p_lo = float(stats.t.sf(t_lo, df))
    p_hi = float(stats.t.cdf(t_hi, df))
    p = max(p_lo, p_hi)
    return {"n_pairs": n, "diff_mean_pt": mean, "diff_sd_pt": sd, "diff_se_pt": se,
            "ci90_pt": [mean - t90 * se, mean + t90 * se], "ci95_pt": [mean - t95 * se, mean + t95 * se],
            "margin_pt": margin, "tost_p_lower": p_lo, "tost_p_upper": p_hi, "tost_p": p,
            "equivalent_at_5pct": bool(p < 0.05),
            # pairs needed for the 90 % interval half-width to reach the margin's distance from the mean
            "pairs_for_equivalence": (int(math.ceil((t90 * sd / (margin - abs(mean))) ** 2))
                                      if abs(mean) < margin else None)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("records", nargs="+")
    ap.add_argument("--margin", type=float, default=1.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    out = []
    for path in a.records:
        rec = json.load(open(path))
        res = tost(paired_diffs(rec), a.margin)
        res.update({"record": path, "protocol": rec.get("protocol", ""), "dropout": rec.get("dropout", ""),
                    "seeds": rec.get("seeds", []), "hip_mean": rec.get("hip_mean"), "ref_mean": rec.get("ref_mean")})
        out.append(res)
        print(f"{path}: {res['dropout']:11s} n={res['n_pairs']:4d} mean {res['diff_mean_pt']:+.2f} pt "
              f"SE {res['diff_se_pt']:.2f}  90% CI [{res['ci90_pt'][0]:+.2f}, {res['ci90_pt'][1]:+.2f}]  "
              f"95% CI [{res['ci95_pt'][0]:+.2f}, {res['ci95_pt'][1]:+.2f}]  TOST p={res['tost_p']:.3g} "
              f"{'EQUIVALENT' if res['equivalent_at_5pct'] else 'not shown'} (need ~{res['pairs_for_equivalence']} pairs)")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
