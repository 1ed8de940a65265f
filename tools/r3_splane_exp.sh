#!/bin/bash
# timing experiment (results invalid in the variants): the s plane's cost -- pass A without its s
# store (nss), and additionally pass E computing s = ws x instead of DMAing the s rows (srec);
# cfg2 (B = 4096) and cfg4 (B = 65536) per-kernel device times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
for lib in libeegnet_hip.so libeegnet_hip_nss.so libeegnet_hip_srec.so; do
  EEGNET_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-folds --no-cfg5 --no-infer > gpurun_out/sx_${lib}_$i.log 2>&1 || { echo BENCH_FAILED $lib; tail -20 gpurun_out/sx_${lib}_$i.log; exit 1; }
  tail -1 gpurun_out/sx_${lib}_$i.log | LIB=$lib python3 -c "
import json,sys,os; d=json.loads(sys.stdin.read()); c=d['cfg4_dp']
print(os.environ['LIB'], 'cfg2 %.3fM %.4f ms' % (d['value']/1e6, d['ms_per_step']), {k: v['avg_us'] for k, v in d['kernels'].items()})
print('   cfg4 %.3fM %.4f ms' % (c['value']/1e6, c['ms_per_step']), {k: v['avg_us'] for k, v in c['kernels'].items()})"
done; done
