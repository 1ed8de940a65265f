#!/bin/bash
# round 3: GPU suite on the current build, then the full bench line (cfg2, folds, cfg5 train, infer) twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_f$i.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_f$i.log; exit 1; }
tail -1 gpurun_out/bench_f$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('cfg2', d['value'], d['ms_per_step'])
for k, v in d.items():
    if isinstance(v, dict) and 'value' in v: print(' ', k, v['value'], v.get('unit'), v.get('ms_per_step'))"
done
