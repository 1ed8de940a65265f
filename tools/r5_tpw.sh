#!/bin/bash
# fold trials-per-workgroup sweep (EEGNET_FOLD_TPW="s,c,b2") at the cfg3 rank shares
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in ${TPWS:-4,8,2 4,4,2 4,2,2 2,8,2 2,4,2 2,2,2}; do
  EPOCHS=3 EEGNET_FOLD_TPW=$t timeout -k 10 120 python -u tools/fold_tpw_sweep.py ${FOLDS:-12 23} 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${TAG:-r5}_tpw.log || { echo SWEEP_FAILED; exit 1; }
done
