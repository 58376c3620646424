#!/usr/bin/env bash
# GPU-box: parity suite, headline bench (with CPU baseline), kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputests_${TAG}.log 2>&1 || { tail -30 gpurun_out/gputests_${TAG}.log; exit 1; }
tail -2 gpurun_out/gputests_${TAG}.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
cat gpurun_out/bench_${TAG}.json &&
rm -rf gpurun_out/prof_${TAG} &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench_${TAG}.json 2> gpurun_out/prof_${TAG}.err &&
python3 tools/trace_summary.py $(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv") > gpurun_out/prof_${TAG}_summary.txt &&
head -20 gpurun_out/prof_${TAG}_summary.txt
