#!/usr/bin/env bash
# Config 5: rocprofv3 kernel stats + cProfile of the host side.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run -- python3 bench.py --config 5 --steps 2 --warmup 1 > gpurun_out/cfg5p.json 2> gpurun_out/cfg5p.err &&
timeout -k 10 600 python -m cProfile -o gpurun_out/cfg5.pstats bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/cfg5c.json 2> gpurun_out/cfg5c.err
rc=$?
find gpurun_out/prof5 -name "*stats*" | head
exit $rc
