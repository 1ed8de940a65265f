#!/bin/bash
# fold trials-per-workgroup sweep over -D builds (libeegnet_hip_t<S><C>.so: EEGNET_FOLD_TPW_S / _C)
# at the cfg3 rank shares; the product library is the 4,8 row
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in ${LIBS:-libeegnet_hip.so libeegnet_hip_t28.so libeegnet_hip_t24.so libeegnet_hip_t38.so libeegnet_hip_t44.so}; do
  echo "== $lib"
  EPOCHS=3 EEGNET_LIB=$lib timeout -k 10 150 python -u tools/fold_tpw_sweep.py ${FOLDS:-12 23 45 90} 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/${TAG:-r6}_tpw.log || { echo SWEEP_FAILED; exit 1; }
done
