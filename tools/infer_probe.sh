#!/bin/bash
# build (here, INFER_PROBE_BUILD=1) or time (GPU) the EEGNET_KX knockout builds of k_infer_bf16_cfg5
set -o pipefail
if [ -n "$INFER_PROBE_BUILD" ]; then
  cd "$(dirname "$0")/.." && mkdir -p eegnetreplication_amd/probe
  for n in ${KXS:-0 1 2 3 4 5}; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -Wno-unused-result \
      -Wno-unused-value -DEEGNET_KX=$n -I include -o eegnetreplication_amd/probe/libeegnet_hip_K$n.so eegnetreplication_amd/csrc/eegnet_kernels.hip &
    while [ $(jobs -r | wc -l) -ge 3 ]; do sleep 2; done
  done
  wait; exit 0
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in ${KXS:-0 1 2 3 4 5}; do
  EEGNET_LIB=probe/libeegnet_hip_K$n.so timeout -k 10 120 python -u tools/infer_probe.py 2>&1 | grep avg_us || { echo PROBE_FAILED $n; exit 1; }
done
