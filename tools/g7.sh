# round 6, call 7: GPU suite subset touching the native tree and fits, configs
# 3/4/5 lines, rank shares after the host-fit and flat-space changes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_tree.py tests/test_gpu_suggest.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_g7.log 2>&1 &&
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/cfg4_g7.err 2>&1 &&
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/cfg5_g7.err 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b6_g7.err 2>&1 &&
timeout -k 10 400 python tools/rank_share.py --config 4 --steps 10 --json gpurun_out/rank_share4_g7.json > gpurun_out/rank_share4_g7.txt 2>&1 &&
timeout -k 10 400 python tools/rank_share.py --config 5 --steps 8 --json gpurun_out/rank_share5_g7.json > gpurun_out/rank_share5_g7.txt 2>&1
