#!/bin/bash
# one GPU call: parity tests, bench, rocprofv3 kernel trace of a short bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
