#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for tw in 512 1024 2048 4096 8192; do
  TPE_TARGET_WORK=$tw timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_$tw.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/sweep_$tw.json')); r=d['roofline']
print($tw, 'p50 %.3f'%d['p50_suggest_ms'], 'above %.4f'%d['stage_ms']['k_above_f32'], 'exec CE/s %.3e'%r['executed_ce_per_s'])"
done
