# round 6, call 4: the whole GPU suite on the round's library, smoke, the
# probe's live-object census, configs 4 / 5 host phases and Python, bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_g4.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_g4.log 2>&1 &&
timeout -k 10 150 python tools/tail_probe.py --steps 2000 --tag g4 > gpurun_out/tail_g4.log 2>&1 &&
timeout -k 10 200 python tools/cfg4_prof.py --config 4 > gpurun_out/cfg4prof_g4.txt 2>&1 &&
timeout -k 10 300 python tools/cfg4_prof.py --config 5 --steps 5 > gpurun_out/cfg5prof_g4.txt 2>&1 &&
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/cfg4_g4.err 2>&1 &&
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/cfg5_g4.err 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b6_drv4.err 2>&1
