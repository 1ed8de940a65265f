#!/bin/bash
# round 3: step timeline with the raw per-workgroup stamps, then the rocprofv3 kernel stats + PMC passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/trace_step.py --dump gpurun_out/stamps_cfg2.npy > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log | grep -E "pass|stamps"
bash tools/profile.sh
