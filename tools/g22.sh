# round 6, call 22: k_fit_main's grid-edge searches (one lane, every wave
# waiting) as a bucket estimate plus exact steps, against the previous kernel
# file; config 5 under the kernel trace, alternating; the fit parity tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2 3; do
  for v in old new; do
    lib=$PWD/hyperopt_amd/libtpe_hip.so
    [ $v = old ] && lib=$PWD/hyperopt_amd/libtpe_hip_old.so
    rm -rf $O/fit_${v}_$r
    TPE_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fit_${v}_$r -o run -- \
        python3 bench.py --config 5 --steps 10 --warmup 1 > $O/fit_${v}_$r.log 2>&1 || { echo "FAILED $v $r"; tail -20 $O/fit_${v}_$r.log; exit 1; }
    echo "$v $r: $(python3 tools/trace_summary.py $(find $O/fit_${v}_$r -name '*kernel_trace.csv') | grep -E 'k_boxes|k_cells_fgt|k_fit_main' | tr -s ' ' | cut -d' ' -f1,9,10 | tr '\n' ';')"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "fit or config5 or order" > $O/tests_g22.log 2>&1; tail -2 $O/tests_g22.log
