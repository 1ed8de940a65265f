#!/bin/bash
# bf16 cfg5 chunked kernel: parity tests, A/B vs the whole-trial kernel; fold sweep; accuracy tool smoke
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_infer.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || { echo BF16_TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/bf16_tests.log | head -30; tail -5 gpurun_out/bf16_tests.log; exit 1; }
tail -1 gpurun_out/bf16_tests.log
for v in 0 1; do
EEGNET_BF16_V1=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-folds --no-cfg5 --no-cfg4 > gpurun_out/bf16_ab_$v.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bf16_ab_$v.log; exit 1; }
tail -1 gpurun_out/bf16_ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['cfg5_infer_bf16']; print('V1=$v', d['value'], d['roofline']['avg_us'], d['roofline']['frac'])"
done
for t in 4,8,2 3,6,2 5,10,2 6,12,3 4,16,2 6,8,2; do
  EEGNET_FOLD_TPW=$t timeout -k 10 120 python -u tools/fold_tpw_sweep.py 90 45 12 >> gpurun_out/fold_sweep2.log 2>&1 || { echo SWEEP_FAILED $t; tail -5 gpurun_out/fold_sweep2.log; exit 1; }
done
grep tpw gpurun_out/fold_sweep2.log
timeout -k 10 300 python -u tools/accuracy_parity.py --protocol ws --epochs 3 --seeds 0 --workers 6 --dropout common --out gpurun_out/acc_smoke_ws.json > gpurun_out/acc_smoke.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_smoke.log; exit 1; }
timeout -k 10 300 python -u tools/accuracy_parity.py --protocol cs --epochs 2 --seeds 0 --workers 6 --dropout independent --cs-folds 0 10 20 --out gpurun_out/acc_smoke_cs.json >> gpurun_out/acc_smoke.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/acc_smoke.log; exit 1; }
grep -v "^  reference" gpurun_out/acc_smoke.log | tail -8
for m in 1 2 4; do for c in 1 2; do
EEGNET_GRIDS_MULT=$m EEGNET_GRIDC_MULT=$c timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-folds --no-cfg5 --no-cfg4 --no-infer > gpurun_out/grid_${m}_${c}.log 2>&1 || { echo GRID_FAILED $m $c; tail -20 gpurun_out/grid_${m}_${c}.log; exit 1; }
tail -1 gpurun_out/grid_${m}_${c}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('grid $m $c', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
done; done
