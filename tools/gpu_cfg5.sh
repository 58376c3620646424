#!/usr/bin/env bash
# Config 5 (1000 dims x 100k history) with the device Parzen fit, plus GPU tests.
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --config 5 --steps 3 --warmup 1 --dims ${DIMS:-1000} > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
rc=$?
tail -30 gpurun_out/pytest_gpu.log; cat gpurun_out/cfg5.json; tail -5 gpurun_out/cfg5.err
exit $rc
