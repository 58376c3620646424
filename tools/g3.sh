# round 6, call 3: the native column store's GPU tests, the RCCL one-rank
# tests, the probe's live-object census, config-4 / config-5 Python profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_devhist.py tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread -k "devhist or rccl or scatter or orders or columns or grid" > gpurun_out/tests_g3.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "incremental or config5" > gpurun_out/tests_g3_cfg5.log 2>&1 &&
timeout -k 10 150 python tools/tail_probe.py --steps 500 --tag g3 > gpurun_out/tail_g3.log 2>&1 &&
timeout -k 10 200 python tools/cfg4_prof.py --config 4 > gpurun_out/cfg4prof_g3.txt 2>&1 &&
timeout -k 10 300 python tools/cfg4_prof.py --config 5 --steps 5 > gpurun_out/cfg5prof_g3.txt 2>&1 &&
timeout -k 10 300 python tools/cfg4_prof.py --config 5 --appending --steps 20 > gpurun_out/cfg5appprof_g3.txt 2>&1
