# round 6, calls 31-32: a k_tables or k_sample_fast variant (the in-tree library,
# 32: the first draws made while the table lands) — the GPU suite on it, then alternating headline lines
# and kernel traces against the previous library (libtpe_hip_base.so)
set -o pipefail
O=gpurun_out
step() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -30 "$log"; exit $rc; fi; }
step 900 $O/g30_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -1 $O/g30_tests.log
for r in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_base.so; else unset TPE_HIP_LIB; fi
    step 300 $O/g30_b_${v}_$r.json python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-config4
    echo "$v $r: $(python -c "import json; d=json.loads(open('$O/g30_b_${v}_$r.json').read().strip().splitlines()[-1]); print(round(d['p50_suggest_ms'],4), round(d['ms_per_step'],4), round(d['p99_suggest_ms'],4), d['stage_ms'])")"
  done
done
for v in base new; do
  if [ $v = base ]; then export TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_base.so; else unset TPE_HIP_LIB; fi
  rm -rf $O/g30_t_$v
  step 300 $O/g30_t_$v.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/g30_t_$v -o run -- python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline --no-config4 --no-quantized --no-appending
  echo "$v trace: $(python3 tools/trace_summary.py $(find $O/g30_t_$v -name '*kernel_trace.csv') | head -3 | awk '{for(i=1;i<=NF;i++) if($i=="med") print $1, $(i+1)}' | tr '\n' ' ')"
done
unset TPE_HIP_LIB
