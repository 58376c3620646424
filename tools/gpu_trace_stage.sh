#!/usr/bin/env bash
# GPU-box: rocprofv3 kernel trace of tools/stage_bench.py (per-kernel durations).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
rm -rf gpurun_out/tprof_${TAG}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof_${TAG} -o run -- \
    python3 tools/stage_bench.py ${REP:-2} > gpurun_out/tprof_${TAG}.txt 2>&1
