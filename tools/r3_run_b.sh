#!/bin/bash
# round 3: full GPU suite (SyncBN stage API, Bn normalisation), train-step timeline, 500-epoch accuracy calibration
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace_step.log 2>&1 || { echo TRACE_STEP_FAILED; tail -20 gpurun_out/trace_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace_step.log
timeout -k 10 700 python -u tools/accuracy_parity.py --protocol ws --epochs 500 --seeds 0 --workers 12 --dropout common --out gpurun_out/acc_ws_e500_s0.json > gpurun_out/acc_ws.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_ws.log; exit 1; }
grep -v "^  reference" gpurun_out/acc_ws.log | tail -5
