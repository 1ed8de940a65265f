# PMC pass: instruction cache behaviour per kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcic; rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || { echo P1_FAIL; tail -5 $OUT/p1.log; exit 1; }
echo PMC_OK
