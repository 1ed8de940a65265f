#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/trace_bf16.py 16384 > gpurun_out/trace_bf16.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/trace_bf16.log; exit 1; }
cat gpurun_out/trace_bf16.log | grep -v amdgpu.ids
