#!/bin/bash
# round 3 profile: rocprofv3 kernel stats + separate PMC passes (tools/profile.sh), bench line with roofline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof
bash tools/profile.sh || exit 1
