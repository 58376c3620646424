# tail probes after the cycle-free documents (round 6): driver-style bench,
# probes at 16 / 14 / 12 host threads, one traced pool, the new GPU test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b6_drv2.err 2>&1 &&
timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag g2def > gpurun_out/tail_g2def.log 2>&1 &&
TPE_HOST_THREADS=14 timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag g2th14 > gpurun_out/tail_g2th14.log 2>&1 &&
TPE_HOST_THREADS=12 timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag g2th12 > gpurun_out/tail_g2th12.log 2>&1 &&
TPE_POOL_TRACE=1 timeout -k 10 150 python tools/tail_probe.py --steps 20 --warmup 2 --tag g2trace > gpurun_out/tail_g2trace.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "more_than_64 or device_fit" > gpurun_out/tests_g2.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread -k "rccl" > gpurun_out/tests_g2_rccl.log 2>&1
