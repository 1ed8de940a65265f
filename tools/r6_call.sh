#!/bin/bash
# Round-6 iteration call: the -m gpu suite on the current build, then (AB=1) the bench A/B of
# libeegnet_hip_base.so (another build beside it) against libeegnet_hip.so (tools/ab.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 800 python -u -m pytest ${TESTS:-tests} -m gpu -v -x --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_gpu_tests.log | sed -e 's/ *\[.*%\]//' | head -30
  tail -1 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; exit 1; }
fi
if [ -n "$AB" ]; then
  bash tools/ab.sh || exit 1
fi
