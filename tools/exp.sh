# time experiment variants of the library: tools/exp.sh libeegnet_hip_NAME.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  EEGNET_LIB=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-infer --no-folds --no-cfg5 --steps 30 --warmup 5 > gpurun_out/bench_exp.log 2>&1 || { tail -20 gpurun_out/bench_exp.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_exp.log').read().strip().splitlines()[-1]);print('$v', d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()})"
done
