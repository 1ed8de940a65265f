#!/bin/bash
# SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE of passes A and E for the product library (lds_step.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ldsc
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/main -o run -- python3 tools/lds_step.py > $OUT/main.log 2>&1 || { echo PMC_FAIL; tail -20 $OUT/main.log; exit 1; }
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
f = glob.glob("gpurun_out/ldsc/main/**/run_counter_collection.csv", recursive=True)[0]
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(f)):
    m = re.search(r"eeg::(k_pass_[a-e])\b", r["Kernel_Name"])
    if m: acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    c = {n: sum(x) / len(x) for n, x in acc[k].items()}
    print(f"{k:10s} conflict {c['SQ_LDS_BANK_CONFLICT']:10.0f} lds_cycles {c['SQ_LDS_IDX_ACTIVE']:11.0f} "
          f"frac {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:6.3f} insts {c['SQ_INSTS_LDS']:10.0f}")
PY
