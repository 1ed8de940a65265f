set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof; mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log | cut -c1-200
