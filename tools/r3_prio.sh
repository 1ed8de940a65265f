#!/bin/bash
# progress-paced issue priority: timeline with per-workgroup stamps, then A/B against the no-priority build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/trace_step.py --dump gpurun_out/stamps_prio.npy > gpurun_out/trace_prio.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_prio.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_prio.log | grep -E "pass"
LIBS="libeegnet_hip_noprio.so libeegnet_hip.so" BENCH_ARGS="--no-cfg4" bash tools/ab.sh
