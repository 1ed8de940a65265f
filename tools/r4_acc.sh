#!/bin/bash
# Accuracy-parity groundwork: the graph-captured reference driver against the
# eager one on a few short units (same accuracies expected up to rounding), then the cross-subject
# learnability of the synthetic-session presets (HIP protocol, 90 folds, 500 epochs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r4acc}
if [ -z "$NOSMOKE" ]; then
for mode in "" "--ref-eager"; do
  timeout -k 10 400 python -u tools/accuracy_parity.py --protocol cs --epochs 20 --seeds 0 --cs-folds 0 40 --workers 2 --dropout common $mode --out gpurun_out/${TAG}_smoke$mode.json > gpurun_out/${TAG}_smoke$mode.log 2>&1 || { echo ACC_SMOKE_FAILED $mode; tail -30 gpurun_out/${TAG}_smoke$mode.log; exit 1; }
  grep -v "^  reference" gpurun_out/${TAG}_smoke$mode.log | tail -2
done
fi
if [ -n "$PRESETS" ]; then
  timeout -k 10 900 python -u tools/synth_cs_sweep.py $PRESETS > gpurun_out/${TAG}_sweep.log 2>&1 || { echo SWEEP_FAILED; tail -30 gpurun_out/${TAG}_sweep.log; exit 1; }
  cat gpurun_out/${TAG}_sweep.log | grep -v warning
fi
