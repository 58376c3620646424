# round 6, call 11: the GPU suite on the one-pass chunked fill, then the
# headline with the fill chunked (default) vs unchunked, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_g11.log 2>&1 &&
for r in 1 2; do
  for v in 2048 100000000; do
    TPE_FILL_CHUNK_MIN=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-quantized --no-config4 --steps 200 --warmup 5 > gpurun_out/ab11_${r}_$v.err 2>&1 || exit 1
    echo "r$r MIN=$v: $(grep -o '"p50_suggest_ms": [0-9.]*\|"mean_suggest_ms": [0-9.]*\|"p50_suggest_ms_appending": [0-9.]*' gpurun_out/ab11_${r}_$v.err | tr '\n' ' ')"
  done
done
