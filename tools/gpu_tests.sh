#!/usr/bin/env bash
# GPU-box: the -m gpu parity suite (library built on the CPU side beforehand).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gputests_${TAG}.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gputests_${TAG}.log | tail -40; exit $rc
