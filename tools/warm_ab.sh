#!/bin/bash
# The headline leg alone at the driver's flags (--steps 20 --warmup 5), fresh process per run,
# alternating survey lengths / warm-ups: how much of the short-run deficit is GPU warm-up
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-infer --no-folds --no-cfg5 --no-cfg4"
for i in 1 2 3; do
  for v in "--steps 20 --warmup 5 --survey 5" "--steps 20 --warmup 5 --survey 20" "--steps 20 --warmup 60 --survey 5" "--steps 100 --warmup 5 --survey 5"; do
    timeout -k 10 120 python -u bench.py $v $Q > gpurun_out/warm.log 2>&1 || { echo FAIL; tail -5 gpurun_out/warm.log; exit 1; }
    echo "$v :: $(tail -1 gpurun_out/warm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3fM %.4f ms k_pass_e %s' % (d['value']/1e6, d['ms_per_step'], (d.get('roofline') or {}).get('avg_us')))")"
  done
done
