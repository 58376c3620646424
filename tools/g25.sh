# round 6, call 25: final evidence on the final library — smoke, GPU suite,
# three driver-style headline runs, kernel trace, PMC passes, config lines,
# config 5 appended under the kernel trace, the N = 2 flow over gloo (two ranks
# on the one GPU)
set -o pipefail
TAG=r06h bash tools/gpu.sh smoke tests &&
TAG=r06h_a BENCH_ARGS="--gpus 1 --steps 20 --warmup 3" bash tools/gpu.sh bench &&
TAG=r06h_b BENCH_ARGS="--gpus 1 --steps 20 --warmup 3" bash tools/gpu.sh bench &&
TAG=r06h_c BENCH_ARGS="--gpus 1 --steps 20 --warmup 3" bash tools/gpu.sh bench &&
TAG=r06h STEPS=50 bash tools/gpu.sh trace pmc &&
TAG=r06h CFG_STEPS=10 bash tools/gpu.sh configs &&
TAG=r06h APP5=--appending CFG_STEPS=10 bash tools/gpu.sh trace5 &&
TAG=r06h REH_CONFIGS=3 CFG_STEPS=5 bash tools/gpu.sh rehearse
