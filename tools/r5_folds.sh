#!/bin/bash
# kernel trace of a 12-fold (cfg3 8-rank share) and a 90-fold epoch: per-kernel time and the gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fgap
for nf in 12 90; do
  EPOCHS=1 timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fgap/kt$nf -o run -- python3 tools/fold_tpw_sweep.py $nf > gpurun_out/fgap/kt$nf.log 2>&1 || { echo KT_FAIL; tail -20 gpurun_out/fgap/kt$nf.log; exit 1; }
  tail -1 gpurun_out/fgap/kt$nf.log
  python3 tools/fold_gaps.py gpurun_out/fgap/kt$nf | tee gpurun_out/fgap/gaps$nf.txt
  rm -f gpurun_out/fgap/kt$nf/*/run_kernel_trace.csv gpurun_out/fgap/kt$nf/run_kernel_trace.csv
done
