#!/bin/bash
# bf16 cfg5: halo-free chunk kernel (r) parity tests, phase trace, A/B against the haloed chunk kernel (c)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_infer.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || { echo BF16_TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/bf16_tests.log | head -30; tail -5 gpurun_out/bf16_tests.log; exit 1; }
tail -1 gpurun_out/bf16_tests.log
for k in r c; do
EEGNET_BF16_KERNEL=$k timeout -k 10 120 python -u tools/trace_bf16.py 16384 > gpurun_out/trace_bf16_$k.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/trace_bf16_$k.log; exit 1; }
echo "== trace $k"; grep -v amdgpu.ids gpurun_out/trace_bf16_$k.log
EEGNET_BF16_KERNEL=$k timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-folds --no-cfg5 --no-cfg4 > gpurun_out/bf16_ab_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bf16_ab_$k.log; exit 1; }
tail -1 gpurun_out/bf16_ab_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['cfg5_infer_bf16']; print('kernel $k', d['value'], d['roofline']['avg_us'], d['roofline']['frac'])"
done
