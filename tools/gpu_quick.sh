#!/bin/bash
# one GPU call: the -m gpu suite (stops at the first failure), then the cfg2 bench line without the
# slow legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|Error|passed|failed" gpurun_out/gpu_tests.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-infer ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
print({k: v["avg_us"] for k, v in d["kernels"].items()})
c = d.get("cfg5_train")
if c: print("cfg5", c["value"], c["ms_per_step"])
print("folds", (d.get("real_protocol_folds") or {}).get("value"))
PY
