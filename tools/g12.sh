# round 6, call 12: evidence on the round's library — smoke, the GPU suite,
# three driver-style headline runs, the kernel trace and the PMC passes
set -o pipefail
TAG=r06 bash tools/gpu.sh smoke tests &&
TAG=r06a bash tools/gpu.sh bench &&
TAG=r06b bash tools/gpu.sh bench &&
TAG=r06c bash tools/gpu.sh bench &&
TAG=r06 STEPS=50 bash tools/gpu.sh trace pmc
