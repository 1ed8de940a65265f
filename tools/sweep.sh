set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for bt in 256 1024 4096 8192; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 --batch $bt > gpurun_out/sweep_b$bt.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sweep_b$bt.log').read().strip().splitlines()[-1]);print('B=$bt',d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
done
