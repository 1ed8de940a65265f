#!/bin/bash
# Round-6 record call: GPU suite + smoke + default bench line + rocprof (tools/r6_round.sh with PROF=1),
# then the bench line at the driver's flags (--steps 20 --warmup 5)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6f}
PROF=1 bash tools/r6_round.sh $TAG || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driverflags.log 2>&1 || { echo BENCH2_FAILED; exit 1; }
tail -1 gpurun_out/${TAG}_bench_driverflags.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver-flags cfg2 %.3fM %.4f ms' % (d['value']/1e6, d['ms_per_step']), 'cfg5', (d.get('cfg5_train') or {}).get('value'), 'folds12', ((d.get('real_protocol_folds') or {}).get('per_share') or {}).get('12'))"
