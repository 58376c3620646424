#!/usr/bin/env bash
# A/B of library variants on one box: bench.py --config $CONFIG per variant in
# LIBS (hyperopt_amd/libtpe_hip_<name>.so; "default" = libtpe_hip.so),
# alternating, ROUNDS times; prints p50 and the device stages per run.
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${LIBS:-default}; do
    if [ "$v" = default ]; then lib=$PWD/hyperopt_amd/libtpe_hip.so; else lib=$PWD/hyperopt_amd/libtpe_hip_$v.so; fi
    out=gpurun_out/ab${CONFIG:-5}_${TAG:-x}_${v}_$r.err
    timeout -k 10 300 env TPE_HIP_LIB=$lib python bench.py --config ${CONFIG:-5} --steps ${STEPS:-10} --warmup 1 \
        ${AB_ARGS:-} > $out 2>&1 || { echo "FAILED $v"; tail -20 $out; exit 1; }
    echo "$v $r: $(grep -o '"p50_step_ms": [0-9.]*\|"stage_ms_per_step": {[^}]*}' $out | tr '\n' ' ')"
  done
done
