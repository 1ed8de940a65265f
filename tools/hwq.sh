#!/bin/bash
# fold-batched leg at several hardware-queue counts (per-process HIP setting)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u -c "
import torch, bench
print($q, bench.bench_folds(torch.device('cuda:0'), 16, 1440, 2))" || exit 1
done
