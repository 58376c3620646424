#!/usr/bin/env bash
# GPU-box bench + kernel-trace profile.  Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
cat gpurun_out/bench_${TAG}.json &&
if [ -z "${NO_PROF:-}" ]; then
  rm -rf gpurun_out/prof_${TAG} &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench_${TAG}.json 2> gpurun_out/prof_${TAG}.err &&
  find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" -exec cat {} \;
fi
