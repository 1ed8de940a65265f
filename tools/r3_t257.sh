#!/bin/bash
# step timeline at 22 x 256 and 22 x 257, B = 2880 (per-phase shader cycles per trial)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for T in 256 257; do
timeout -k 10 120 python -u tools/trace_step.py --batch 2880 --T $T > gpurun_out/trace_t$T.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/trace_t$T.log; exit 1; }
echo "== T=$T"; grep -v amdgpu.ids gpurun_out/trace_t$T.log | grep -E "^pass|phases"
done
