"""Where a fold-indexed train step's time goes: per-kernel durations and the idle gaps between
consecutive dispatches, from a rocprofv3 kernel trace of tools/fold_tpw_sweep.py.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/fold_tpw_sweep.py 12
    python tools/fold_gaps.py DIR
"""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    f = glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "eeg::" in r["Kernel_Name"]]
    # EPOCHS=1: a warm-up epoch, then the timed one (the second half of the eeg:: dispatches)
    rows = rows[len(rows) // 2:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    prev = None
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[n].append((e - s) / 1e3)
        if prev is not None:
            gap[n].append((s - prev) / 1e3)
        prev = e
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print(f"{len(rows)} dispatches, span {span:.1f} us, kernels busy {busy:.1f} us, gaps {span - busy:.1f} us")
    for n, v in dur.items():
        g = gap.get(n, [0.0])
        print(f"{n:48s} n {len(v):5d} avg {sum(v) / len(v):7.2f} us  gap before avg {sum(g) / len(g):6.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
