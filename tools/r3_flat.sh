#!/bin/bash
# one-level (flat) reduction only for grids <= 128: timeline, then A/B against the current build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EEGNET_LIB=libeegnet_hip_trflat128.so timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_flat.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_flat.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_flat.log | grep -E "^pass"
LIBS="libeegnet_hip_flat128.so libeegnet_hip.so" BENCH_ARGS="--no-cfg4 --no-cfg5" bash tools/ab.sh
