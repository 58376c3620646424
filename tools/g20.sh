# round 6, call 20: final evidence on the final library — smoke, GPU suite,
# three driver-style headline runs, kernel trace, PMC passes, config lines, and
# config 5 appended under the kernel trace (no framework kernels)
set -o pipefail
TAG=r06f bash tools/gpu.sh smoke tests &&
TAG=r06f_a BENCH_ARGS="--gpus 1 --steps 20 --warmup 3" bash tools/gpu.sh bench &&
TAG=r06f_b BENCH_ARGS="--gpus 1 --steps 20 --warmup 3" bash tools/gpu.sh bench &&
TAG=r06f_c BENCH_ARGS="--gpus 1 --steps 20 --warmup 3" bash tools/gpu.sh bench &&
TAG=r06f STEPS=50 bash tools/gpu.sh trace pmc &&
TAG=r06f CFG_STEPS=10 bash tools/gpu.sh configs &&
TAG=r06f APP5=--appending CFG_STEPS=10 bash tools/gpu.sh trace5
