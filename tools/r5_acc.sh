#!/bin/bash
# One chunk of the accuracy-parity runs per gpurun call (round 5: reference workers with one HW queue
# each and no product import, tools/accuracy_parity.py --worker-hw-queues):
#   PROTO=cs|ws SEEDS="3" DROP=common|independent FOLDS="45 ... 89" (cs only) WORKERS=12
#   tools/r5_acc.sh TAG     -> gpurun_out/TAG.json, TAG.log (merge chunks with tools/acc_merge.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-acc}
FARGS=""
[ "$PROTO" = "cs" ] && FARGS="--cs-folds $FOLDS"
timeout -k 10 ${LIMIT:-1120} python -u tools/accuracy_parity.py --protocol ${PROTO:-cs} --epochs ${EPOCHS:-500} \
  --seeds ${SEEDS:-0} --workers ${WORKERS:-12} --worker-hw-queues ${HWQ:-1} --dropout ${DROP:-common} $FARGS \
  --out gpurun_out/$TAG.json > gpurun_out/$TAG.log 2>&1 || { echo ACC_FAILED; tail -20 gpurun_out/$TAG.log; exit 1; }
grep -v -E "^  (reference|waiting)" gpurun_out/$TAG.log | tail -8
