#!/bin/bash
# GPU suite on the current build; timeline of the RGB 32 / 16-group reduction variant; A/B against it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log | grep -E "^pass|stamps"
EEGNET_LIB=libeegnet_hip_trg16.so timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_g16.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_g16.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_g16.log | grep -E "^pass|stamps"
LIBS="libeegnet_hip_g16.so libeegnet_hip.so" BENCH_ARGS="--no-cfg4" bash tools/ab.sh
