# round 6, call 16: driver-style headline runs on the 2-ms pool spin, then the
# other configs' lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/drv16_$r.err 2>&1 || exit 1
  grep '^{' gpurun_out/drv16_$r.err > gpurun_out/drv16_$r.json
  python - gpurun_out/drv16_$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print('value %.3e p50 %.4f p99 %.4f mean %.4f ms_per_step %.4f steps %s cpu %.3g app %.4f q %.4f' % (
    d['value'], d['p50_suggest_ms'], d['p99_suggest_ms'], d['mean_suggest_ms'], d['ms_per_step'],
    d['tail']['steps_ms'][:4], d['cpu_baseline']['value'], d['p50_suggest_ms_appending'], d['quantized_branch']['p50_suggest_ms']))
PY
done
TAG=r06 CFG_STEPS=10 bash tools/gpu.sh configs &&
timeout -k 10 600 python bench.py --config 5 --appending --steps 20 --warmup 2 > gpurun_out/cfg5app_r06.err 2>&1 &&
grep '^{' gpurun_out/cfg5app_r06.err
