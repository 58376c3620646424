#!/usr/bin/env bash
# GPU-box: gpu tests, then per-stage device times and the headline bench with the
# default flags and with TPE_DEBUG_FLAGS=$AB_FLAGS (A/B of a batch option).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/gputests_${TAG}.log 2>&1 || { grep -E "PASSED|FAILED|ERROR|Error|assert" gpurun_out/gputests_${TAG}.log | tail -30; exit 1; }
  tail -2 gpurun_out/gputests_${TAG}.log
fi
timeout -k 10 300 python tools/stage_bench.py ${REP:-20} > gpurun_out/stage_${TAG}.txt 2>&1 &&
TPE_DEBUG_FLAGS=${AB_FLAGS:-0} timeout -k 10 300 python tools/stage_bench.py ${REP:-20} > gpurun_out/stage_${TAG}_ab.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
TPE_DEBUG_FLAGS=${AB_FLAGS:-0} timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/bench_${TAG}_ab.json 2> gpurun_out/bench_${TAG}_ab.err &&
grep -h -o '"p50_suggest_ms": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_${TAG}.json gpurun_out/bench_${TAG}_ab.json
