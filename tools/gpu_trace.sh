#!/usr/bin/env bash
# GPU-box: rocprofv3 kernel trace + stats of a short headline bench run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
rm -rf gpurun_out/prof_${TAG}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/prof_bench_${TAG}.json 2> gpurun_out/prof_${TAG}.err &&
cat gpurun_out/prof_bench_${TAG}.json
