#!/bin/bash
# Round-6 (session 4) call: the wide-path GPU tests on the product build, then the alternating bench A/B
# of LIBS (tools/ab.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6b}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v -x --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" gpurun_out/${TAG}_gpu_tests.log | head -30
  tail -1 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || { echo "TESTS rc=$rc"; exit 1; }
fi
bash tools/ab.sh
