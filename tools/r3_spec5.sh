#!/bin/bash
# cfg5 wide kernels with compile-time cfg5 geometry (SPEC): wide / parity / protocol GPU tests, cfg5 train leg x2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-folds --no-cfg4 --no-infer > gpurun_out/spec5_$i.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/spec5_$i.log; exit 1; }
tail -1 gpurun_out/spec5_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cfg5_train']; print('cfg2', d['value'], '| cfg5 train', c['value'], c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
done
