#!/bin/bash
# round 3: parity suite subset (train step paths), step timeline, cfg2 + folds bench legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log | grep -E "pass|prologue stamps"
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-cfg5 --no-infer --no-cfg4 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('cfg2', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})
print('folds', d['real_protocol_folds']['value'])
"
