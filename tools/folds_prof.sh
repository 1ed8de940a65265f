#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fprof
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-infer --no-cfg5 --no-cfg4 > gpurun_out/fprof/kt.log 2>&1 || { echo KT_FAIL; tail -20 gpurun_out/fprof/kt.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/fprof/kt/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "eeg::" in n:
        print(f"{n[:60]:60s} calls {r['Calls']:>6} avg_us {float(r['AverageNs'])/1e3:8.2f} tot_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
rm -f gpurun_out/fprof/kt/run_kernel_trace.csv
