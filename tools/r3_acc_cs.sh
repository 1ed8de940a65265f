#!/bin/bash
# accuracy parity, cross-subject protocol (p = 0.25), reference's 500 epochs, 5 seeds, one fold per test
# subject (repeat 1: 0-based folds 0, 10, ..., 80), common dropout masks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1130 python -u tools/accuracy_parity.py --protocol cs --epochs 500 --seeds 0 1 2 3 4 --workers 15 --dropout common --cs-folds 0 10 20 30 40 50 60 70 80 --out gpurun_out/acc_cs_e500_s5_common.json > gpurun_out/acc_cs5.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_cs5.log; exit 1; }
grep -v "^  reference" gpurun_out/acc_cs5.log | tail -8
