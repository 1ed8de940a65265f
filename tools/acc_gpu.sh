#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_protocols.py || exit 1
timeout -k 10 900 python -u tools/accuracy_parity.py --epochs 100 --seeds 0 1 2 --p 0.5 --out gpurun_out/acc_p05.json 2>&1 | tee gpurun_out/acc_p05.log
