# round 6, call 34: final evidence on the final library — smoke, GPU suite,
# three headline runs with the driver's own arguments, kernel trace, PMC
# passes, config lines, config 5 appended under the kernel trace, the N = 2
# flow over gloo, and the N = 8 rank shares of configs 5 and 4
set -o pipefail
TAG=r06j bash tools/gpu.sh smoke tests &&
TAG=r06j_a BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu.sh bench &&
TAG=r06j_b BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu.sh bench &&
TAG=r06j_c BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu.sh bench &&
TAG=r06j STEPS=50 bash tools/gpu.sh trace pmc &&
TAG=r06j CFG_STEPS=10 bash tools/gpu.sh configs &&
TAG=r06j APP5=--appending CFG_STEPS=10 bash tools/gpu.sh trace5 &&
TAG=r06j REH_CONFIGS=3 CFG_STEPS=5 bash tools/gpu.sh rehearse &&
timeout -k 10 300 python tools/rank_share.py --config 5 --steps 8 --only-n 8 > gpurun_out/rank8_5_r06j.txt 2>&1 &&
timeout -k 10 300 python tools/rank_share.py --config 4 --steps 10 --only-n 8 > gpurun_out/rank8_4_r06j.txt 2>&1
