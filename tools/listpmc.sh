cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1; echo rc=$?
grep -c . gpurun_out/pmc_list.txt
