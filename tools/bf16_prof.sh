#!/bin/bash
# bf16 tests + bench line + kernel-trace stats of the inference leg (which instantiation ran)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/bf16.sh || exit 1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt5 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-folds > gpurun_out/kt5.log 2>&1 || { echo KT_FAIL; tail -20 gpurun_out/kt5.log; exit 1; }
rm -f gpurun_out/kt5/run_kernel_trace.csv
cut -d, -f1-4 gpurun_out/kt5/run_kernel_stats.csv | head -4
