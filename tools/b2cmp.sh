#!/bin/bash
# pass C/D variants at B=4096: one-trial-per-wave (default) vs whole-trial block-2 kernels (EEGNET_B2=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A="--no-cpu-baseline --no-infer --no-folds --no-cfg5 --steps 30"
timeout -k 10 200 python -u bench.py $A > gpurun_out/b2_0.log 2>&1 || exit 1
EEGNET_B2=1 timeout -k 10 200 python -u bench.py $A > gpurun_out/b2_1.log 2>&1 || exit 1
for f in gpurun_out/b2_0.log gpurun_out/b2_1.log; do python - "$f" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["ms_per_step"], {k:v["avg_us"] for k,v in d["kernels"].items()})
PY
done
