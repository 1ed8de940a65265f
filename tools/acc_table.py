"""DESIGN §7.1's accuracy table from the merged round-4 records (profiles/r4_accuracy_*.json):
one markdown row per protocol / dropout mode.

    python tools/acc_table.py profiles/r4_accuracy_cs_e500_s3_common.json ...
"""
import json
import sys


def main():
    print("| Run | pairs | HIP | reference | paired diff | 95 % CI | identical pairs |")
    print("|---|---|---|---|---|---|---|")
    for p in sys.argv[1:]:
        r = json.load(open(p))
        name = ("cross-subject, p = 0.25" if r["protocol"].startswith("cross") else "within-subject, p = 0.5")
        print(f"| {name}, {r['epochs']} epochs, seeds {','.join(map(str, r['seeds']))}, {r['dropout']} masks "
              f"(`{p}`) | {r['n_pairs']} | {r['hip_mean']:.2f} % | {r['ref_mean']:.2f} % | "
              f"{r['diff_mean_pt']:+.2f} pt (SE {r['diff_se_pt']:.2f}) | "
              f"[{r['ci95_pt'][0]:+.2f}, {r['ci95_pt'][1]:+.2f}] | {r['pairs_identical']} |")


if __name__ == "__main__":
    main()
