#!/bin/bash
# fold-launch TPW fine sweep + accuracy tool smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in 4,8,2 3,6,2 5,10,2 6,12,3 4,16,2 4,8,1 6,8,2; do
  EEGNET_FOLD_TPW=$t timeout -k 10 120 python -u tools/fold_tpw_sweep.py 90 45 12 >> gpurun_out/fold_sweep2.log 2>&1 || { echo SWEEP_FAILED $t; tail -5 gpurun_out/fold_sweep2.log; exit 1; }
done
grep tpw gpurun_out/fold_sweep2.log
timeout -k 10 300 python -u tools/accuracy_parity.py --protocol ws --epochs 3 --seeds 0 --workers 6 --dropout common --out gpurun_out/acc_smoke_ws.json > gpurun_out/acc_smoke.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_smoke.log; exit 1; }
timeout -k 10 300 python -u tools/accuracy_parity.py --protocol cs --epochs 2 --seeds 0 --workers 6 --dropout independent --cs-folds 0 10 20 --out gpurun_out/acc_smoke_cs.json >> gpurun_out/acc_smoke.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_smoke.log; exit 1; }
tail -8 gpurun_out/acc_smoke.log
