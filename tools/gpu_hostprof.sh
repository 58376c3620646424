#!/usr/bin/env bash
# GPU-box: gpu tests, headline bench, the host-side cProfile breakdown of the
# headline suggest (tools/host_profile.py) and its profiler-free split
# (tools/host_split.py).  The library is built on the
# CPU side beforehand (it travels in-tree).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/gputests_${TAG}.log 2>&1 || { tail -30 gpurun_out/gputests_${TAG}.log; exit 1; }
  tail -3 gpurun_out/gputests_${TAG}.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
cat gpurun_out/bench_${TAG}.json &&
timeout -k 10 300 python tools/host_profile.py ${STEPS:-30} > gpurun_out/hostprof_${TAG}.txt 2>&1 &&
head -c 3000 gpurun_out/hostprof_${TAG}.txt &&
timeout -k 10 300 python tools/host_split.py 200 > gpurun_out/hostsplit_${TAG}.txt 2>&1 &&
cat gpurun_out/hostsplit_${TAG}.txt
