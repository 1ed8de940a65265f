#!/bin/bash
# Round-4 measurement call: the step timeline of the traced build, the x-statistics-table A/B at
# B = 4096, then (ACC=1) tools/r4_acc.sh's accuracy groundwork (PRESETS: learnability sweep).
#   tools/r4_probe.sh TAG   -> gpurun_out/TAG_*
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r4p}
if [ -z "$NOTRACE" ]; then
  timeout -k 10 240 python -u tools/trace_step.py > gpurun_out/${TAG}_timeline.txt 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${TAG}_timeline.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_timeline.txt
fi
if [ -z "$NOXS" ]; then
  timeout -k 10 300 python -u tools/xstat_ab.py > gpurun_out/${TAG}_xstat_ab.log 2>&1 || { echo XSTAT_AB_FAILED; tail -20 gpurun_out/${TAG}_xstat_ab.log; exit 1; }
  cat gpurun_out/${TAG}_xstat_ab.log
fi
if [ -n "$ACC" ]; then
  bash tools/r4_acc.sh ${TAG}acc || exit 1
fi
