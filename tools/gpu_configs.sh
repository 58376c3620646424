#!/usr/bin/env bash
# Measure BASELINE.json configs 1, 2, 4, 5 on one GPU (config 3 is bench.py's default).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 1 --steps 5 --warmup 1 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err &&
timeout -k 10 300 python bench.py --config 2 --steps 30 --warmup 3 > gpurun_out/cfg2.json 2> gpurun_out/cfg2.err &&
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 > gpurun_out/cfg4.json 2> gpurun_out/cfg4.err &&
timeout -k 10 600 python bench.py --config 5 --steps 2 --warmup 1 ${CFG5_ARGS:-} > gpurun_out/cfg5.json 2> gpurun_out/cfg5.err
rc=$?
cat gpurun_out/cfg*.json; tail -n 3 gpurun_out/cfg*.err
exit $rc
