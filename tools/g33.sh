# round 6, call 35: more of the final library's headline runs with the
# driver's arguments (another box), and its 2000-step tail probe
set -o pipefail
for s in d e f; do
  TAG=r06k_$s BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash tools/gpu.sh bench || exit 1
done
timeout -k 10 400 python tools/tail_probe.py --steps 2000 --warmup 5 --tag final_lib > gpurun_out/g33_tail.log 2>&1 && tail -2 gpurun_out/g33_tail.log
