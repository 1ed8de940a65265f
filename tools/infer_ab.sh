#!/bin/bash
# k_infer_bf16_cfg5 time per launch for several builds (LIBS, in eegnetreplication_amd/), alternating, one call
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  for lib in ${LIBS:-libeegnet_hip_base.so libeegnet_hip.so}; do
    EEGNET_LIB=$lib timeout -k 10 120 python -u tools/infer_probe.py 2>&1 | grep avg_us || { echo PROBE_FAILED $lib; exit 1; }
  done
done
