#!/bin/bash
# GPU test call: the -m gpu suite (or the files given as arguments), without -x so one call reports
# every failure; a hang ends at the per-test timeout and names its test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FILES="${@:-tests}"
timeout -k 10 900 python -u -m pytest $FILES -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|XFAIL|SKIPPED" gpurun_out/gpu_tests.log | sed -e 's/ *\[.*%\]//' | tail -120
tail -3 gpurun_out/gpu_tests.log
exit $rc
