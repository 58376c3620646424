# round 6, call 13: driver-style headline runs with the CPU baseline after the
# GPU measurements (bench.CpuBaselineChild)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/drv13_$r.err 2>&1 || exit 1
  grep '^{' gpurun_out/drv13_$r.err > gpurun_out/drv13_$r.json
  python - gpurun_out/drv13_$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print('value %.3e p50 %.4f p99 %.4f mean %.4f ms_per_step %.4f steps %s cpu %.3g app %.4f' % (
    d['value'], d['p50_suggest_ms'], d['p99_suggest_ms'], d['mean_suggest_ms'], d['ms_per_step'],
    d['tail']['steps_ms'][:5], d['cpu_baseline']['value'], d['p50_suggest_ms_appending']))
PY
done
