set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for v in default TPE_POOL_SPIN_US=50 TPE_POOL_SPIN_US=0 TPE_HOST_THREADS=8; do
  if [ "$v" = default ]; then e=""; else e="$v"; fi
  timeout -k 10 300 env $e python bench.py --no-cpu-baseline > gpurun_out/ab_${v}_$r.out 2> gpurun_out/ab_${v}_$r.err || exit 1
  echo "$r $v $(grep -o '"p50_suggest_ms": [0-9.]*\|"p99_suggest_ms": [0-9.]*' gpurun_out/ab_${v}_$r.out | head -2 | tr '\n' ' ')"
done
done
