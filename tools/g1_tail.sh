set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b6_drv1.err 2>&1 &&
timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag def > gpurun_out/tail_def.log 2>&1 &&
TPE_POOL_SPIN_US=50 timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag spin50 > gpurun_out/tail_spin50.log 2>&1 &&
TPE_HOST_THREADS=4 timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag th4 > gpurun_out/tail_th4.log 2>&1 &&
timeout -k 10 150 python tools/tail_probe.py --steps 3000 --nogc --tag nogc > gpurun_out/tail_nogc.log 2>&1 &&
TPE_HOST_THREADS=8 timeout -k 10 150 python tools/tail_probe.py --steps 3000 --tag th8 > gpurun_out/tail_th8.log 2>&1 &&
cat /sys/fs/cgroup/cpu.max > gpurun_out/cpumax.txt; nproc >> gpurun_out/cpumax.txt; cat /sys/fs/cgroup/cpu.stat >> gpurun_out/cpumax.txt; true
