"""Merge accuracy_parity.py result files of one protocol / dropout mode run in chunks (fold subsets,
seed subsets: one gpurun call each) into one record with the paired statistics over all units.

    python tools/acc_merge.py OUT.json IN1.json IN2.json ...
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from accuracy_parity import summarize  # noqa: E402


def main():
    out, ins = sys.argv[1], sys.argv[2:]
    recs = [json.load(open(p)) for p in ins]
    keys = {(r["epochs"], r["dropout"], r["protocol"].split(",")[0]) for r in recs}
    assert len(keys) == 1, f"mixed runs: {keys}"
    pairs, runs, folds = [], [], []
    for r, p in zip(recs, ins):
        for run in r["runs"]:
            runs.append(dict(run, source=os.path.basename(p)))
            pairs += list(zip(run["hip"], run["ref"]))
        folds.append(r["protocol"])
    res = {"protocol": recs[0]["protocol"].split(",")[0], "chunks": folds, "data": recs[0]["data"],
           "epochs": recs[0]["epochs"], "dropout": recs[0]["dropout"],
           "seeds": sorted({run["seed"] for run in runs}), "runs": runs,
           "hip_mean": float(np.mean([h for h, _ in pairs])), "ref_mean": float(np.mean([r for _, r in pairs]))}
    res.update(summarize(pairs))
    res["within_1pt"] = bool(-1.0 <= res["ci95_pt"][0] and res["ci95_pt"][1] <= 1.0)
    res["wall_s"] = round(sum(r.get("wall_s", 0.0) for r in recs), 1)
    per_seed = {}
    for run in runs:
        per_seed.setdefault(run["seed"], ([], []))
        per_seed[run["seed"]][0].extend(run["hip"])
        per_seed[run["seed"]][1].extend(run["ref"])
    res["per_seed"] = {str(s): {"units": len(h), "hip_mean": float(np.mean(h)), "ref_mean": float(np.mean(r))}
                       for s, (h, r) in sorted(per_seed.items())}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("runs", "chunks")}))


if __name__ == "__main__":
    main()
