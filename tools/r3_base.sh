#!/bin/bash
# round 3 baseline: full GPU test suite, smoke, default bench line, rocprofv3 kernel stats + HBM PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c 1-400
[ -n "$NOPROF" ] && exit 0
bash tools/profile.sh
