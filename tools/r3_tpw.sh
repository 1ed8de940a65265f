#!/bin/bash
# fold-launch trials per workgroup sweep (streaming passes s, block-2 passes c), 90 folds, 8 epochs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for s in 2 4 8; do for c in 4 8 16; do
  EPOCHS=8 EEGNET_FOLD_TPW=$s,$c,2 timeout -k 10 120 python -u tools/fold_tpw_sweep.py 90 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/tpw $s,$c: /" || { echo SWEEP_FAILED; exit 1; }
done; done
