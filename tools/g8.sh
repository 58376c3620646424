# round 6, call 8: the shard axes' tests, per-rank shares, config 5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_devhist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_g8.log 2>&1 &&
timeout -k 10 400 python tools/rank_share.py --config 4 --steps 10 --json gpurun_out/rank_share4_g8.json > gpurun_out/rank_share4_g8.txt 2>&1 &&
timeout -k 10 400 python tools/rank_share.py --config 5 --steps 8 --json gpurun_out/rank_share5_g8.json > gpurun_out/rank_share5_g8.txt 2>&1 &&
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/cfg5_g8.err 2>&1 &&
timeout -k 10 300 python bench.py --config 5 --appending --steps 20 --warmup 2 > gpurun_out/cfg5app_g8.err 2>&1
