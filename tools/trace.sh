set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python -u tools/trace_step.py "$@" > gpurun_out/trace.log 2>&1; rc=$?; cat gpurun_out/trace.log; exit $rc
