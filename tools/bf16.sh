# GPU iteration for the bf16 eval kernel: its parity tests, then a bench line (train + cfg5 infer legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_infer.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/bf16_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|mismatch|PASSED" gpurun_out/bf16_tests.log | head -40; tail -5 gpurun_out/bf16_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/bf16_tests.log | tail -15
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step']);print(d['cfg5_infer_bf16'])"
