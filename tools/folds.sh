#!/bin/bash
# GPU iteration for FoldBatch: its tests, then a bench line with the folds leg (no CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_folds.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/folds_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED" gpurun_out/folds_tests.log | head -30; tail -5 gpurun_out/folds_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/folds_tests.log | tail -5
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --no-infer > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['value']);print(d['real_protocol_folds'])"
