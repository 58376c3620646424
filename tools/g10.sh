# round 6, call 10: per-rank shares on the current library; the packer's
# sections (TPE_PACK_TRACE variant) and the tree marks at N = 8
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/rank_share.py --config 4 --steps 10 --json gpurun_out/rank_share4_g10.json > gpurun_out/rank_share4_g10.txt 2>&1 &&
timeout -k 10 400 python tools/rank_share.py --config 5 --steps 8 --json gpurun_out/rank_share5_g10.json > gpurun_out/rank_share5_g10.txt 2>&1 &&
TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_ptrace.so TPE_TREE_TRACE=1 timeout -k 10 300 python tools/rank_share.py --config 5 --steps 8 --only-n 8 > gpurun_out/ptrace5_g10.txt 2> gpurun_out/ptrace5_g10.err &&
TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_ptrace.so TPE_TREE_TRACE=1 timeout -k 10 300 python tools/rank_share.py --config 4 --steps 8 --only-n 8 > gpurun_out/ptrace4_g10.txt 2> gpurun_out/ptrace4_g10.err
