# round 6, call 33: the N > 1 bench flow rehearsed with 4 and 8 ranks on the
# box's one GPU (gloo: RCCL takes one rank per device) — config 3 (the driver's
# scaling run) at 4 and 8, configs 4 and 5 at 8
set -o pipefail
O=gpurun_out
step() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -30 "$log"; exit $rc; fi; }
for spec in "4 3" "8 3" "8 4" "8 5"; do
  set -- $spec; n=$1; c=$2
  step 600 $O/g31_reh_n${n}_c${c}.err env TPE_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + 10 * n + c)) bench.py --gpus $n --config $c \
      --steps 5 --warmup 2 --no-cpu-baseline --no-quantized --no-appending
  grep '^{' $O/g31_reh_n${n}_c${c}.err > $O/g31_reh_n${n}_c${c}.json
  python -c "import json; d=json.loads(open('$O/g31_reh_n${n}_c${c}.json').read().strip().splitlines()[-1]); print('N=$n config $c', '%.3e' % d['value'], round(d['ms_per_step'], 4), d.get('scaling'), d['config'].get('parallelism'))"
done
