# round 6, call 17: GPU suite after the dict-type and record-reuse changes;
# config 5's appended step by section; config 4 / 5-appending lines
set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_g17.log 2>&1 &&
tail -2 gpurun_out/tests_g17.log &&
timeout -k 10 300 python tools/cfg5_app_sections.py --steps 30 > gpurun_out/cfg5_sections_g17.txt 2>&1 &&
cat gpurun_out/cfg5_sections_g17.txt &&
timeout -k 10 600 python bench.py --config 5 --appending --steps 20 --warmup 2 > gpurun_out/cfg5app_g17.err 2>&1 &&
timeout -k 10 600 python bench.py --config 4 --steps 10 --warmup 1 > gpurun_out/cfg4_g17.err 2>&1 &&
python - <<'PY'
import json
for f in ('gpurun_out/cfg5app_g17.err', 'gpurun_out/cfg4_g17.err'):
    d = [json.loads(l) for l in open(f) if l.startswith('{')][0]
    print(f, d['p50_step_ms'], d.get('p50_step_ms_dict_results'), d['host_phases_us'])
PY

timeout -k 10 300 python tools/rank_share.py --config 4 --steps 10 --only-n 8 > gpurun_out/rank8_g17.txt 2>&1 && grep -v amdgpu gpurun_out/rank8_g17.txt
