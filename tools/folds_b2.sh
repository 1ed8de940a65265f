#!/bin/bash
# real-protocol folds leg: block-2 passes C / D as whole-trial 256-thread workgroups (default at
# small per-launch grids) vs one trial per wave (EEGNET_B2=0), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A="--no-cpu-baseline --no-infer --no-cfg5 --no-profile --steps 5 --warmup 2"
for i in 1 2; do
  for v in dflt 0; do
    if [ $v = dflt ]; then timeout -k 10 200 python -u bench.py $A > gpurun_out/fb_$v.log 2>&1 || exit 1
    else EEGNET_B2=$v timeout -k 10 200 python -u bench.py $A > gpurun_out/fb_$v.log 2>&1 || exit 1; fi
    python - gpurun_out/fb_$v.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "folds", d["real_protocol_folds"]["value"])
PY
  done
done
