"""Per-kernel means of the PMC passes of tools_pmc.sh (gpurun_out/pmc/p*), per launch."""
import csv
import os
import re
import sys
from collections import defaultdict

src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "pmc")
acc = defaultdict(lambda: defaultdict(list))
for d in sorted(os.listdir(src)):
    f = os.path.join(src, d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for row in csv.DictReader(open(f)):
        m = re.search(r"eeg::(k_\w+)", row["Kernel_Name"])
        if m:
            acc[m.group(1)][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    cs = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(k)
    for c in sorted(cs):
        print(f"   {c:28s} {cs[c]:16.0f}")
