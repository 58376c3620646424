# round 6, call 27: the fit's box parts (tpe_fit_job.fgt_n) — the new GPU test
# first, then the GPU suite, then config 5 with the parts (TPE_FGT_FUSED=1)
# against the rows read back (0), alternating, and a config-5 kernel trace
set -o pipefail
O=gpurun_out
step() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -30 "$log"; exit $rc; fi; }
step 300 $O/g27_boxtest.log python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "box_parts or box_moment"
grep -E "PASSED|FAILED|passed|failed" $O/g27_boxtest.log | tail -8
step 900 $O/g27_tests.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
tail -2 $O/g27_tests.log
for r in 1 2; do
  for f in 1 0; do
    TPE_FGT_FUSED=$f step 300 $O/g27_cfg5_f${f}_$r.json python bench.py --config 5 --steps 10 --warmup 2
    echo "fused=$f run $r: $(python -c "import json; d=json.loads(open('$O/g27_cfg5_f${f}_$r.json').read().strip().splitlines()[-1]); print(round(d['p50_step_ms'],4), d['stage_ms_per_step'])")"
  done
done
rm -rf $O/g27_trace5
step 600 $O/g27_trace5.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/g27_trace5 -o run -- python3 bench.py --config 5 --steps 10 --warmup 2
python3 tools/trace_summary.py $(find $O/g27_trace5 -name "*kernel_trace.csv") > $O/g27_trace5_summary.txt
head -14 $O/g27_trace5_summary.txt
