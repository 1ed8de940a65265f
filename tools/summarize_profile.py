"""Turn a tools_profile.sh run (gpurun_out/prof) into the committed profile summaries:

    profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary, as written
    profiles/<tag>_pmc_summary.json   per-kernel mean of every PMC counter over the dispatches
    profiles/pmc_traffic.json         HBM bytes per launch for the pass kernels (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md 'HBM': FETCH_SIZE (KB) is doubled on gfx950 (wide coalesced
reads are tallied at half their bytes); WRITE_SIZE (KB) is taken as-is.
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    m = re.search(r"eeg::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:60]


def main(tag, src=os.path.join(ROOT, "gpurun_out", "prof")):
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"),
                os.path.join(out, f"{tag}_kernel_stats.csv"))
    acc = defaultdict(lambda: defaultdict(list))
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc") or not os.path.exists(f):
            continue
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    summ = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    with open(os.path.join(out, f"{tag}_pmc_summary.json"), "w") as fh:
        json.dump(summ, fh, indent=1, sort_keys=True)
    traffic = {}
    for k, cs in summ.items():
        if not k.startswith("k_") or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = 2.0 * cs["FETCH_SIZE"] * 1024
        wr = cs["WRITE_SIZE"] * 1024
        traffic[k] = {"hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd),
                      "write_bytes": round(wr), "source": f"profiles/{tag}_pmc_summary.json"}
    with open(os.path.join(out, "pmc_traffic.json"), "w") as fh:
        json.dump(traffic, fh, indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
