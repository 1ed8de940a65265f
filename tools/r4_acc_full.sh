#!/bin/bash
# One chunk of the 500-epoch accuracy-parity runs per gpurun call:
#   PROTO=cs|ws SEEDS="0 1 2" DROP=common|independent FOLDS="0 1 ... 44" (cs only) WORKERS=15
#   tools/r4_acc_full.sh TAG     -> gpurun_out/TAG.json, TAG.log (merge chunks with tools/acc_merge.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-acc}
FARGS=""
[ "$PROTO" = "cs" ] && FARGS="--cs-folds $FOLDS"
timeout -k 10 ${LIMIT:-1120} python -u tools/accuracy_parity.py --protocol ${PROTO:-cs} --epochs ${EPOCHS:-500} \
  --seeds ${SEEDS:-0} --workers ${WORKERS:-15} --dropout ${DROP:-common} $FARGS --out gpurun_out/$TAG.json \
  > gpurun_out/$TAG.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/$TAG.log; exit 1; }
grep -v -E "^  (reference|waiting)" gpurun_out/$TAG.log | tail -6
