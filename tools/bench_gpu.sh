#!/bin/bash
# bench.py (default line) + rocprofv3 kernel-trace stats of a short bench run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 500 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("value", d["value"], "ms/step", d["ms_per_step"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d["kernels"].items(): print("  ", k, v)
c = d.get("cfg5_train")
if c:
    print("cfg5", c["value"], c["ms_per_step"], c["step_fp32_frac"], c["roofline"]["kernel"], c["roofline"]["frac"])
    for k, v in c["kernels"].items(): print("  ", k, v)
print("infer", d["cfg5_infer_bf16"]["value"] if d.get("cfg5_infer_bf16") else None)
print("folds", d.get("real_protocol_folds"))
print("cpu", d.get("cpu_baseline"))
PY
if [ -n "$PROF" ]; then
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-folds > gpurun_out/prof/kt.log 2>&1 || { echo KT_FAIL; tail -20 gpurun_out/prof/kt.log; exit 1; }
find gpurun_out/prof -name "*stats*"
rm -f gpurun_out/prof/kt/run_kernel_trace.csv
fi
