# build experiment variants of the trace library: tools/build_exp.sh NAME -DFLAG ...
# -> eegnetreplication_amd/libeegnet_hip_NAME.so (select with EEGNET_LIB=libeegnet_hip_NAME.so)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared ${SLP_FLAG--fno-slp-vectorize} -Wno-unused-result \
  -Wno-unused-value ${TRACE_FLAG--DEEGNET_TRACE} "$@" -I include -o eegnetreplication_amd/libeegnet_hip_$name.so \
  eegnetreplication_amd/csrc/eegnet_kernels.hip
