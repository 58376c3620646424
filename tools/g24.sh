# round 6, call 24: config 4's sample pass at two workgroups a CU with four
# candidates a lane (TPE_FAST_WPC2=1) against three with two (default),
# alternating; bench lines and the kernel trace's k_sample_fast
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
  for v in 0 1; do
    rm -rf $O/np_${v}_$r
    TPE_FAST_WPC2=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/np_${v}_$r -o run -- \
        python3 bench.py --config 4 --steps 10 --warmup 1 > $O/np_${v}_$r.log 2>&1 || { echo "FAILED $v $r"; tail -20 $O/np_${v}_$r.log; exit 1; }
    echo "WPC2=$v $r: p50 $(grep -o '"p50_step_ms": [0-9.]*' $O/np_${v}_$r.log) $(python3 tools/trace_summary.py $(find $O/np_${v}_$r -name '*kernel_trace.csv') | grep -E 'k_sample_fast|k_tables' | tr -s ' ' | cut -d' ' -f1,2,9,10 | tr '\n' ';')"
  done
done
