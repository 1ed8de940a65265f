#!/bin/bash
# Round 5: the persistent step (k_step) on the GPU -- the -m gpu suite, then the cfg2 bench leg with
# k_step (default) and with the five-launch step (EEGNET_PERSIST=0), alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r5p}
mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_gpu_tests.log | sed -e 's/ *\[.*%\]//' | head -30
  tail -1 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit 1; }
fi
for i in 1 2; do
  for P in 1 0; do
    EEGNET_PERSIST=$P timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-infer --no-folds --no-cfg5 --no-cfg4 --steps 50 > gpurun_out/${TAG}_bench_p${P}_$i.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/${TAG}_bench_p${P}_$i.log; exit 1; }
    tail -1 gpurun_out/${TAG}_bench_p${P}_$i.log | P=$P python3 -c "
import json,sys,os; d=json.loads(sys.stdin.read())
print('persist', os.environ['P'], 'cfg2 %.3fM %.4f ms' % (d['value']/1e6, d['ms_per_step']), 'loss', d['final_loss'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
  done
done
