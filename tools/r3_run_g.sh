#!/bin/bash
# round 3: GPU suite, step timeline, bench line twice (cfg2, folds, cfg5 train)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log | grep -E "^pass|stamps"
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-infer --no-cfg4 > gpurun_out/bench_g$i.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_g$i.log; exit 1; }
tail -1 gpurun_out/bench_g$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['cfg5_train']
print('cfg2', d['value'], d['ms_per_step'], '| folds', d['real_protocol_folds']['value'], '| cfg5', c['value'], c['ms_per_step'], {k: v['avg_us'] for k, v in c['kernels'].items()})"
done
