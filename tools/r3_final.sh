#!/bin/bash
# round 3 final: GPU suite, smoke, step timeline, the default bench line (all legs, CPU baseline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log | grep -E "^pass"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('cfg2', d['value'], d['ms_per_step'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'], 'cpu', d['cpu_baseline'])
for k, v in d.items():
    if isinstance(v, dict) and 'value' in v and k != 'cpu_baseline': print(' ', k, v['value'], v.get('ms_per_step'))"
