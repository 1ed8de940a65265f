#!/bin/bash
# round 3: bf16 eval phase trace, train-step timeline, 500-epoch accuracy calibration (one seed, WS)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/trace_bf16.py 16384 > gpurun_out/trace_bf16.log 2>&1 || { echo TRACE_BF16_FAILED; tail -20 gpurun_out/trace_bf16.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_bf16.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log
timeout -k 10 900 python -u tools/accuracy_parity.py --protocol ws --epochs 500 --seeds 0 --workers 12 --dropout common --out gpurun_out/acc_ws_e500_s0.json > gpurun_out/acc_ws.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_ws.log; exit 1; }
grep -v "^  reference" gpurun_out/acc_ws.log | tail -5
