#!/bin/bash
# rocprofv3: kernel trace + stats, then separate PMC passes (one counter group per run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --no-folds --no-cfg4"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc1 -o run -- $B > $OUT/pmc1.log 2>&1 || { echo PMC1_FAIL; tail -20 $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- $B > $OUT/pmc2.log 2>&1 || { echo PMC2_FAIL; tail -20 $OUT/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- $B > $OUT/pmc3.log 2>&1 || { echo PMC3_FAIL; tail -20 $OUT/pmc3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc4 -o run -- $B > $OUT/pmc4.log 2>&1 || { echo PMC4_FAIL; tail -20 $OUT/pmc4.log; exit 1; }
find $OUT -name "*.csv" | head -20
rm -f $OUT/kt/run_kernel_trace.csv   # per-dispatch rows: large, the stats file is what is kept
