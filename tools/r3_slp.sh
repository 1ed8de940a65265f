#!/bin/bash
# SLP-vectorised build (packed FP32 FMAs) against the current one: bench legs with per-kernel times
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBS="libeegnet_hip_slp.so libeegnet_hip.so" BENCH_ARGS="--no-cfg4" bash tools/ab.sh
