#!/bin/bash
# round 3, first GPU call: full GPU test suite, smoke, default bench line, fold-launch TPW sweep
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c 1-600
for t in 13,32,6 8,16,4 4,8,2 2,4,1 16,32,8 1,1,1; do
  EEGNET_FOLD_TPW=$t timeout -k 10 120 python -u tools/fold_tpw_sweep.py 90 36 12 >> gpurun_out/fold_sweep.log 2>&1 || { echo SWEEP_FAILED $t; tail -5 gpurun_out/fold_sweep.log; exit 1; }
done
cat gpurun_out/fold_sweep.log
