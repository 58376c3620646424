# round 6, call 14: where the first timed suggests after a short warm-up go
# (tail_probe: per-step host phases), warm-up 3 vs 30
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/tail_probe.py --steps 40 --warmup 3 --tag w3 > gpurun_out/tail_w3.log 2>&1 &&
timeout -k 10 300 python tools/tail_probe.py --steps 40 --warmup 30 --tag w30 > gpurun_out/tail_w30.log 2>&1 &&
python - <<'PY'
import json
for t in ('w3', 'w30'):
    d = json.load(open('gpurun_out/tail_%s.json' % t))
    print(t, 'p50', d['summary']['p50_us'], 'phases', d['summary']['phase_names'])
    for r in d['rows'][:8]:
        print('  step', r['i'], r['wall_us'], r['ph'], 'run', r['run_us'], 'wait', r['wait_us'], 'gc', r['gc'])
PY
