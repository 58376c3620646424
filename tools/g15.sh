# round 6, call 15: the first timed suggest after warm-up 3 — pool spin 200 us
# (default) vs 2 ms, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for sp in 200 2000; do
    TPE_POOL_SPIN_US=$sp timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sp15_${r}_$sp.err 2>&1 || exit 1
    python - gpurun_out/sp15_${r}_$sp.err $sp <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]
print('spin %s: p50 %.4f p99 %.4f mean %.4f ms_per_step %.4f first %s cg %s' % (sys.argv[2], d['p50_suggest_ms'], d['p99_suggest_ms'],
      d['mean_suggest_ms'], d['ms_per_step'], d['tail']['steps_ms'][:4],
      {k: d['tail']['cgroup_cpu_stat_warmup_and_timed'].get(k) for k in ('usage_usec', 'nr_throttled')}))
PY
  done
done
