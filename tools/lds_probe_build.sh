#!/bin/bash
# knockout builds for tools/lds_probe.sh: eegnetreplication_amd/probe/libeegnet_hip_{E,A}<n>.so
cd "$(dirname "$0")/.."
OUT=eegnetreplication_amd/probe
mkdir -p $OUT
jobs_=()
for v in ${VARIANTS:-E0 E1 E2 E3 E4 E5 E6 E7 A1 A3 A5 A6 A7}; do
  p=${v:0:1}; n=${v:1}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fno-slp-vectorize -Wno-unused-result \
    -Wno-unused-value -DEEGNET_LDSX_$p=$n -I include -o $OUT/libeegnet_hip_$v.so eegnetreplication_amd/csrc/eegnet_kernels.hip &
  while [ $(jobs -r | wc -l) -ge 4 ]; do sleep 2; done
done
wait
ls $OUT
