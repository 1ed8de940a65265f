#!/bin/bash
# Round 6 GPU call: the -m gpu suite, smoke, the default bench line, then the rocprofv3 kernel trace and
# PMC passes of tools/profile.sh (outputs gpurun_out/TAG_*, gpurun_out/prof/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r6}
mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_gpu_tests.log | sed -e 's/ *\[.*%\]//' | head -30
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
print('folds', f.get('value'), f.get('per_share'))
print('cfg5', c.get('value'), {k: v['avg_us'] for k, v in (c.get('kernels') or {}).items()}, 'infer', i.get('value'), (i.get('roofline') or {}).get('frac'))
print('eval2', (d.get('cfg2_eval_fp32') or {}).get('value'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
fi
if [ -n "$PROF" ]; then
  bash tools/profile.sh || { echo PROFILE_FAILED; exit 1; }
  echo PROFILE_OK
fi
