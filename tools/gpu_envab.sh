#!/usr/bin/env bash
# GPU-box: headline p50 + stage times for each "NAME=VALUE" environment setting in ENVS
# ("-" = none).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r01}
i=0
for e in ${ENVS:--}; do
  i=$((i+1))
  if [ "$e" = "-" ]; then e=TPE_NONE=1; fi
  env "$e" timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-100} > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || exit 1
  echo "$e: $(grep -o '"p50_suggest_ms": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_${TAG}_$i.json | tr '\n' ' ')"
done
