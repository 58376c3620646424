# round 6, call 19: config 5 appended after the record reuse; GPU suite subset
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
step() {  # limit log cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED ($rc): $*"; tail -30 "$log"; exit $rc; fi
}
step 300 $O/cfg5_sections_g19.txt python tools/cfg5_app_sections.py --steps 30
cat $O/cfg5_sections_g19.txt
step 600 $O/cfg5app_g19.err python bench.py --config 5 --appending --steps 20 --warmup 2
step 600 $O/cfg5_g19.err python bench.py --config 5 --steps 10 --warmup 1
python - <<'PY'
import json
for f in ('gpurun_out/cfg5app_g19.err', 'gpurun_out/cfg5_g19.err'):
    d = [json.loads(l) for l in open(f) if l.startswith('{')][0]
    print(f, d['p50_step_ms'], d['host_phases_us'], d['stage_ms_per_step'])
PY
step 900 $O/tests_g19.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_native_tree.py tests/test_gpu_devhist.py -x -q --timeout 300 --timeout-method thread
tail -2 $O/tests_g19.log
