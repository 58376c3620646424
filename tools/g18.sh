# round 6, call 18: GPU suite (batched dicts typed as numpy's; remote entries
# in the results pass), config 5's appended step by section, config 4 / 5
# lines, per-rank shares of configs 4 and 5
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
step 900 $O/tests_g18.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 $O/tests_g18.log
step 300 $O/cfg5_sections_g18.txt python tools/cfg5_app_sections.py --steps 30
cat $O/cfg5_sections_g18.txt
step 600 $O/cfg5app_g18.err python bench.py --config 5 --appending --steps 20 --warmup 2
step 600 $O/cfg4_g18.err python bench.py --config 4 --steps 10 --warmup 1
python - <<'PY'
import json
for f in ('gpurun_out/cfg5app_g18.err', 'gpurun_out/cfg4_g18.err'):
    d = [json.loads(l) for l in open(f) if l.startswith('{')][0]
    print(f, d['p50_step_ms'], d.get('p50_step_ms_dict_results'), d['host_phases_us'])
PY
step 400 $O/rank_share4_g18.txt python tools/rank_share.py --config 4 --steps 10 --json $O/rank_share4_g18.json
step 400 $O/rank_share5_g18.txt python tools/rank_share.py --config 5 --steps 8 --json $O/rank_share5_g18.json
grep -v amdgpu $O/rank_share4_g18.txt $O/rank_share5_g18.txt
