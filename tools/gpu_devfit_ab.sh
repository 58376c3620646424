#!/usr/bin/env bash
# GPU-box A/B: headline bench with the default device-fit threshold and with
# TPE_DEVICE_FIT_MIN=$DFM (continuous above mixtures fitted on the device).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab_default_${TAG}.json 2>/dev/null &&
TPE_DEVICE_FIT_MIN=${DFM:-1024} timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab_devfit_${TAG}.json 2>/dev/null &&
timeout -k 10 200 python tools/stage_bench.py 20 > gpurun_out/stage_${TAG}.txt 2>&1 &&
TPE_DEVICE_FIT_MIN=${DFM:-1024} timeout -k 10 200 python tools/stage_bench.py 20 > gpurun_out/stage_devfit_${TAG}.txt 2>&1 &&
python -c "
import json
for f in ('default', 'devfit'):
    d = json.load(open('gpurun_out/ab_%s_${TAG}.json' % f)); print(f, 'p50 %.3f ms' % d['p50_suggest_ms'], 'value %.3e' % d['value'], {k: round(v*1e3,1) for k, v in d['stage_ms'].items()})
" && cat gpurun_out/stage_${TAG}.txt gpurun_out/stage_devfit_${TAG}.txt
