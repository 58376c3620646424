# round 6, call 21: config 5's table stage — k_boxes with two row pairs
# prefetched and k_cells_fgt's box-to-Taylor sums one Hermite function at a
# time (new), at 4 (default) / 5 / 6 waves a SIMD, against the previous kernel
# file (old); alternating, config 5 under the kernel trace; then the config
# parity tests on the new library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
  for v in old new w5 w6; do
    lib=$PWD/hyperopt_amd/libtpe_hip.so
    [ $v != new ] && lib=$PWD/hyperopt_amd/libtpe_hip_$v.so
    rm -rf $O/boxes_${v}_$r
    TPE_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/boxes_${v}_$r -o run -- \
        python3 bench.py --config 5 --steps 10 --warmup 1 > $O/boxes_${v}_$r.log 2>&1 || { echo "FAILED $v $r"; tail -20 $O/boxes_${v}_$r.log; exit 1; }
    echo "$v $r: $(python3 tools/trace_summary.py $(find $O/boxes_${v}_$r -name '*kernel_trace.csv') | grep -E 'k_boxes|k_cells_fgt|k_fit_main' | tr -s ' ' | cut -d' ' -f1,9,10 | tr '\n' ';')"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests_g21.log 2>&1; tail -2 $O/tests_g21.log
