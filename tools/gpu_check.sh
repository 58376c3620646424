#!/usr/bin/env bash
# GPU-box check: build, smoke, GPU tests.  Every GPU step has its own time limit
# and the steps are chained so the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/smoke.log; tail -30 gpurun_out/pytest_gpu.log
exit $rc
