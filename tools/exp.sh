# time experiment variants of the library: tools/exp.sh libeegnet_hip_NAME.so ...
# (EXP_CFG5=1: also the cfg5 training leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
X="--no-cfg5"; [ -n "$EXP_CFG5" ] && X=""
for v in "$@"; do
  EEGNET_LIB=$v timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-infer --no-folds $X --steps 30 --warmup 5 > gpurun_out/bench_exp.log 2>&1 || { tail -20 gpurun_out/bench_exp.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/bench_exp.log').read().strip().splitlines()[-1])
print('$v', d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['kernels'].items()})
c=d.get('cfg5_train')
if c: print('   cfg5', c['value'], c['ms_per_step'], {k:v['avg_us'] for k,v in c['kernels'].items()})"
done
