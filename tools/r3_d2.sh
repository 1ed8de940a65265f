#!/bin/bash
# pass D at two 8-wave workgroups per CU (<= 128 VGPRs, grid x2) against the current build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EEGNET_LIB=libeegnet_hip_d2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/d2_tests.log 2>&1 || { echo D2_TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/d2_tests.log | head -20; }
tail -1 gpurun_out/d2_tests.log
LIBS="libeegnet_hip_d2.so libeegnet_hip.so" BENCH_ARGS="--no-cfg4 --no-cfg5" bash tools/ab.sh
