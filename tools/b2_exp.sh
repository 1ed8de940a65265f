#!/bin/bash
# experiment: narrow C/D as whole-trial block-2 workgroups (EEGNET_B2=1) vs one trial per wave
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_tests.sh tests/test_gpu_folds.py tests/test_gpu_parity.py || exit 1
EEGNET_B2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coverage.py tests/test_gpu_folds.py tests/test_gpu_distributed.py -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_b2.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_b2.log; grep -E "^E " gpurun_out/gpu_tests_b2.log | head -5
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--no-cpu-baseline --no-infer --no-cfg5 --steps 30" bash tools/bench_gpu.sh || exit 1
cp gpurun_out/bench.json gpurun_out/bench_default.json
EEGNET_B2=1 BENCH_ARGS="--no-cpu-baseline --no-infer --no-cfg5 --steps 30" bash tools/bench_gpu.sh
