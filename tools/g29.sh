# round 6, call 29 (and 30): k_boxes variants (29: powers in two half-length chains; 30: rows through three LDS-DMA stages)
# (libtpe_hip_ab.so) against the final library, alternating config-5 kernel
# traces; the box-moment parity test on the variant first
set -o pipefail
O=gpurun_out
step() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -30 "$log"; exit $rc; fi; }
TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_ab.so step 300 $O/g29_boxtest.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread -k "box_moment or config5"
grep -E "PASSED|FAILED|passed|failed" $O/g29_boxtest.log | tail -8
for r in 1 2; do
  for v in base ab; do
    rm -rf $O/g29_t_${v}_$r
    if [ $v = ab ]; then export TPE_HIP_LIB=$PWD/hyperopt_amd/libtpe_hip_ab.so; else unset TPE_HIP_LIB; fi
    step 300 $O/g29_t_${v}_$r.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/g29_t_${v}_$r -o run -- python3 bench.py --config 5 --steps 10 --warmup 2
    echo "$v run $r: $(python3 tools/trace_summary.py $(find $O/g29_t_${v}_$r -name '*kernel_trace.csv') | grep -E 'k_boxes|k_cells_fgt|k_fit_main' | awk '{print $1, $(NF-3)}' | tr '\n' ' ')"
  done
done
unset TPE_HIP_LIB
