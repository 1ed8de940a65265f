# PMC passes over a short bench run: VALU/LDS/MFMA activity per kernel (one counter group per run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc; mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || { echo P1_FAIL; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_DATA_FIFO_FULL --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 || { echo P2_FAIL; tail -5 $OUT/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_CYCLES SQ_WAVES --output-format csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1 || { echo P3_FAIL; tail -5 $OUT/p3.log; exit 1; }
echo PMC_OK
