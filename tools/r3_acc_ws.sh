#!/bin/bash
# accuracy parity, within-subject protocol, reference's 500 epochs, 5 seeds, common dropout masks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/accuracy_parity.py --protocol ws --epochs 500 --seeds 0 1 2 3 4 --workers 14 --dropout common --out gpurun_out/acc_ws_e500_s5_common.json > gpurun_out/acc_ws5.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_ws5.log; exit 1; }
grep -v "^  reference" gpurun_out/acc_ws5.log | tail -8
