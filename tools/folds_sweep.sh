#!/bin/bash
# real-protocol fold-batch leg at several fold counts (bench.py --folds N, cfg2 leg trimmed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for nf in ${NFS:-16 32 48}; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-infer --no-cfg5 --no-profile --folds $nf > gpurun_out/folds_$nf.log 2>&1 || { echo FAIL $nf; tail -5 gpurun_out/folds_$nf.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/folds_$nf.log').read().strip().splitlines()[-1]); f=d['real_protocol_folds']; print($nf, f['value'], f.get('per_fold_streams_graphed_value'), f.get('sequential_folds_value'))"
done
