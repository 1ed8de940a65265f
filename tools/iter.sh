# one GPU iteration: parity tests, then the step timeline and a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED|mismatch" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u tools/trace_step.py > gpurun_out/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/trace.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
