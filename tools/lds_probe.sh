#!/bin/bash
# SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE of passes A and E per knockout build (lds_probe_build.sh):
# the drop against build E0 (= the product source) is that access class's share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ldsp
mkdir -p $OUT
for v in ${VARIANTS:-E0 E1 E2 E3 E4 E5 E6 E7 A1 A3 A5 A6 A7}; do
  EEGNET_LIB=probe/libeegnet_hip_$v.so timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d $OUT/$v -o run -- python3 tools/lds_step.py > $OUT/$v.log 2>&1 || { echo PMC_FAIL $v; tail -20 $OUT/$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, re
from collections import defaultdict
print(f"{'build':6s} {'kernel':10s} {'conflict':>10s} {'lds_cycles':>11s} {'frac':>6s} {'lds_insts':>10s}")
for d in sorted(glob.glob("gpurun_out/ldsp/*/")):
    v = d.rstrip("/").split("/")[-1]
    f = glob.glob(d + "**/run_counter_collection.csv", recursive=True)
    if not f: continue
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        m = re.search(r"eeg::(k_pass_[ae])\b", r["Kernel_Name"])
        if m: acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        c = {n: sum(x) / len(x) for n, x in acc[k].items()}
        print(f"{v:6s} {k:10s} {c['SQ_LDS_BANK_CONFLICT']:10.0f} {c['SQ_LDS_IDX_ACTIVE']:11.0f} "
              f"{c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:6.3f} {c['SQ_INSTS_LDS']:10.0f}")
PY
