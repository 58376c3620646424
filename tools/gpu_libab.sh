#!/usr/bin/env bash
# GPU-box: stage times and headline p50 for each library variant named in LIBS
# (hyperopt_amd/libtpe_hip_<name>.so; "default" = libtpe_hip.so).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r01}
for v in ${LIBS:-default}; do
  if [ "$v" = default ]; then lib=$PWD/hyperopt_amd/libtpe_hip.so; else lib=$PWD/hyperopt_amd/libtpe_hip_$v.so; fi
  TPE_HIP_LIB=$lib timeout -k 10 300 python tools/stage_bench.py ${REP:-20} > gpurun_out/stage_${TAG}_$v.txt 2>&1 || exit 1
  TPE_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/bench_${TAG}_$v.json 2> gpurun_out/bench_${TAG}_$v.err || exit 1
  echo "$v: $(grep -o '"p50_suggest_ms": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_${TAG}_$v.json | tr '\n' ' ')"
done
