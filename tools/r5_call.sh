#!/bin/bash
# One GPU call of round 5: every -m gpu test (no -x: one call reports every failure), smoke(), the
# default bench line, then (AB=1) an A/B of the bench's cfg2 leg against the library + Python trees
# of earlier revisions extracted under abtrees/ (each tree drives its own library), alternating.
# Usage: tools/r4_call.sh TAG   (outputs gpurun_out/TAG_*)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r4}
mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|SKIPPED" gpurun_out/${TAG}_gpu_tests.log | sed -e 's/ *\[.*%\]//' | head -40
  tail -1 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit 1; }
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); f=d.get('real_protocol_folds') or {}; c=d.get('cfg5_train') or {}; i=d.get('cfg5_infer_bf16') or {}
print('cfg2 %.3fM %.4f ms' % (d['value']/1e6, d['ms_per_step']), 'roof', (d.get('roofline') or {}).get('kernel'), (d.get('roofline') or {}).get('frac'))
print('kernels', {k: v['avg_us'] for k, v in d['kernels'].items()})
print('folds', f.get('value'), f.get('per_share'), f.get('predicted_scaling'))
print('cfg5', c.get('value'), 'infer', i.get('value'), (i.get('roofline') or {}).get('frac'))
print('cpu', (d.get('cpu_baseline') or {}).get('value'), [(l['cores'], l['value']) for l in (d.get('cpu_baseline') or {}).get('legs', [])])"
fi
if [ -n "$AB" ]; then
  for i in 1 2; do
    for tree in ${TREES:-abtrees/r3g abtrees/r3end .}; do
      ( cd $tree && timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-infer --no-folds --no-cfg5 --no-cfg4 --steps 50 ) > gpurun_out/${TAG}_ab_$(basename $tree)_$i.log 2>&1 || { echo AB_FAILED $tree; tail -20 gpurun_out/${TAG}_ab_$(basename $tree)_$i.log; exit 1; }
      tail -1 gpurun_out/${TAG}_ab_$(basename $tree)_$i.log | TREE=$tree python3 -c "
import json,sys,os; d=json.loads(sys.stdin.read())
print(os.environ['TREE'], 'cfg2 %.3fM %.4f ms' % (d['value']/1e6, d['ms_per_step']), {k: v['avg_us'] for k, v in d['kernels'].items()})"
    done
  done
fi
