# round 6, call 5: measured per-rank shares of configs 4 and 5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/rank_share.py --config 4 --steps 10 --json gpurun_out/rank_share4_g5.json > gpurun_out/rank_share4_g5.txt 2>&1 &&
timeout -k 10 400 python tools/rank_share.py --config 5 --steps 8 --json gpurun_out/rank_share5_g5.json > gpurun_out/rank_share5_g5.txt 2>&1
