#!/usr/bin/env bash
# GPU-box: steady-state per-stage device times (tools/stage_bench.py).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 300 python tools/stage_bench.py ${REP:-20} > gpurun_out/stage_${TAG}.txt 2>&1; rc=$?
cat gpurun_out/stage_${TAG}.txt; exit $rc
