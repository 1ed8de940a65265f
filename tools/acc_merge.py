"""Merge accuracy_parity.py result files of one protocol / dropout mode run in chunks (fold subsets,
seed subsets: one gpurun call each) into one record with the paired statistics over all units.

    python tools/acc_merge.py OUT.json IN1.json IN2.json[:SEED,SEED...] ...

A ":0,1" suffix keeps only those seeds' runs of that input (a seed cut off by a time limit and rerun
whole in another chunk).
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from accuracy_parity import summarize  # noqa: E402


def main():
    out, args = sys.argv[1], sys.argv[2:]
    ins, keep = [], []
    for a in args:
        path, _, seeds = a.partition(":")
        ins.append(path)
        keep.append({int(x) for x in seeds.split(",")} if seeds else None)
    recs = [json.load(open(p)) for p in ins]
    keys = {(r["epochs"], r["dropout"], r["protocol"].split(",")[0]) for r in recs}
    assert len(keys) == 1, f"mixed runs: {keys}"
    pairs, runs, folds, seen = [], [], [], set()
    for r, p, k in zip(recs, ins, keep):
        for run in r["runs"]:
            if k is not None and run["seed"] not in k:
                continue
            for u in run["units"]:
                key = (r["protocol"], run["seed"], u)
                assert key not in seen, f"unit merged twice: {key}"
                seen.add(key)
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
