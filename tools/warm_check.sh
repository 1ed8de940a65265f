#!/bin/bash
# The full default bench line at the driver's flags, three fresh processes (MIN_UNTIMED in effect)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/r6zd_bench_$i.log 2>&1 || { echo FAIL; tail -5 gpurun_out/r6zd_bench_$i.log; exit 1; }
  tail -1 gpurun_out/r6zd_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; f=d.get('real_protocol_folds') or {}; c=d.get('cfg5_train') or {}; print('cfg2 %.3fM %.4f ms untimed %s roof %s %s us %s | cfg5 %s | folds %s 12: %s' % (d['value']/1e6, d['ms_per_step'], d.get('untimed_steps'), r.get('kernel'), r.get('avg_us'), r.get('frac'), c.get('value'), f.get('value'), (f.get('per_share') or {}).get('12')))"
done
