#!/bin/bash
# A/B of two builds of the library in one GPU call: libeegnet_hip_base.so (built from another
# revision, copied beside the current one) against libeegnet_hip.so, alternating, bench legs only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq 1 ${ITERS:-2}); do
  for lib in ${LIBS:-libeegnet_hip_base.so libeegnet_hip.so}; do
    EEGNET_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-infer ${BENCH_ARGS} > gpurun_out/ab_${lib}_$i.log 2>&1 || { echo BENCH_FAILED $lib; tail -20 gpurun_out/ab_${lib}_$i.log; exit 1; }
    LIB=$lib python - <<'PY'
import json, os
d = json.loads(open(f"gpurun_out/ab_{os.environ['LIB']}_1.log" if False else max((f"gpurun_out/{f}" for f in os.listdir("gpurun_out") if f.startswith("ab_" + os.environ["LIB"])), key=os.path.getmtime)).read().strip().splitlines()[-1])
c = d.get("cfg5_train") or {}
print(os.environ["LIB"], "cfg2 %.3fM" % (d["value"] / 1e6), "cfg5 %.4fM" % (c.get("value", 0) / 1e6),
      "folds %.3fM" % ((d.get("real_protocol_folds") or {}).get("value", 0) / 1e6),
      {k: v["avg_us"] for k, v in (c.get("kernels") or {}).items()},
      {k: v["avg_us"] for k, v in (d.get("kernels") or {}).items()})
PY
  done
done
