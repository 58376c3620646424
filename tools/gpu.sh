#!/usr/bin/env bash
# One runner for every GPU-box task (the library is built on the CPU side
# beforehand and travels in-tree).  Usage:
#
#   tools/gpu.sh TASK [TASK ...]        tasks run in order; the first failure ends the script
#
#   tests      -m gpu parity suite                       (PYTEST_ARGS; PYTEST_K = one -k expression)
#   smoke      __graft_entry__.smoke()
#   bench      headline bench.py                         (BENCH_ARGS)
#   trace      rocprofv3 --kernel-trace --stats of a short headline bench run (BENCH_ARGS)
#   pmc        PMC counter passes on the headline bench, one rocprofv3 run per group
#   stage      steady-state per-stage device times        (REP)
#   configs    bench.py --config 1, 2, 4, 5 (CONFIGS)
#   rehearse   bench.py --gpus 2 over gloo, two ranks on the one GPU (REH_CONFIGS)
#   hostsplit  host-side time split of the headline suggest
#   phases     tools/phase_prof.py per workload (PHASE_WL) under the kernel trace
#   nativesplit native fits / tpe_suggest_tree / device stages of the headline suggest
#   hostprof   cProfile of the headline suggest on the device
#   app5       config 5 appending: cProfile + bench line (STEPS, CFG_STEPS)
#   cfgprof    cProfile of one step of config CONFIG (default 5)
#   pmcloop    PMC counter passes on tools/suggest_loop.py (the real suggest flow)
#   apitrace   HIP API + kernel + copy trace of tools/suggest_loop.py -> timeline of the last suggests
#   counters   rocprofv3 -L (the counters this box offers) -> gpurun_out/counters.txt
#   libab      stage times + headline p50 per library variant in LIBS
#              (hyperopt_amd/libtpe_hip_<name>.so; "default" = libtpe_hip.so)
#
# Outputs go to gpurun_out/<task>_<TAG>.*; every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out

step() {  # limit_seconds logfile cmd...
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "FAILED ($rc): $*"; tail -40 "$log"
    exit $rc
  fi
}

prof_run() {  # name counters...
  local name=$1; shift
  rm -rf $O/pmc_${TAG}/$name
  step 300 $O/pmc_${TAG}/$name.log rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
      -d $O/pmc_${TAG}/$name -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-quantized --no-appending --no-config4 ${BENCH_ARGS:-}
}

for task in "$@"; do
  case $task in
    tests)
      step 900 $O/tests_${TAG}.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"}
      grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests_${TAG}.log | tail -60 ;;
    smoke)
      step 300 $O/smoke_${TAG}.log python -c "import __graft_entry__ as g; g.smoke()"
      tail -3 $O/smoke_${TAG}.log ;;
    bench)
      step 600 $O/bench_${TAG}.err python bench.py ${BENCH_ARGS:-}
      grep '^{' $O/bench_${TAG}.err > $O/bench_${TAG}.json; cat $O/bench_${TAG}.json ;;
    trace)
      rm -rf $O/trace_${TAG}
      step 600 $O/trace_${TAG}.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_${TAG} -o run -- \
          python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-quantized --no-appending --no-config4 ${BENCH_ARGS:-}
      python3 tools/trace_summary.py $(find $O/trace_${TAG} -name "*kernel_trace.csv") > $O/trace_${TAG}_summary.txt
      head -25 $O/trace_${TAG}_summary.txt ;;
    pmc)
      mkdir -p $O/pmc_${TAG}
      prof_run fetch FETCH_SIZE
      prof_run write WRITE_SIZE
      prof_run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
      prof_run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU
      if [ -n "${PMC_EXTRA:-}" ]; then prof_run extra $PMC_EXTRA; fi
      python3 tools/pmc_summary.py $O/pmc_${TAG} > $O/pmc_${TAG}/summary.json
      python3 -c "import json; print(json.dumps(json.load(open('$O/pmc_${TAG}/summary.json'))['traffic'], indent=1))" ;;
    stage)
      step 300 $O/stage_${TAG}.txt python tools/stage_bench.py ${REP:-20}
      cat $O/stage_${TAG}.txt ;;
    configs)
      for c in ${CONFIGS:-1 2 4 5}; do
        step 600 $O/cfg${c}_${TAG}.err python bench.py --config $c --steps ${CFG_STEPS:-5} --warmup 1
        grep '^{' $O/cfg${c}_${TAG}.err > $O/cfg${c}_${TAG}.json; cat $O/cfg${c}_${TAG}.json
      done ;;
    envab)
      # stage times + headline p50 per environment setting in ENVAB (space-separated
      # VAR=value specs, "default" = none), alternating on one box
      for v in ${ENVAB:-default}; do
        if [ "$v" = default ]; then e=""; else e="$v"; fi
        step 300 $O/stage_${TAG}_$v.txt env $e python tools/stage_bench.py ${REP:-20}
        step 300 $O/bench_${TAG}_$v.err env $e python bench.py --no-cpu-baseline --no-quantized --no-config4 --steps 100
        echo "$v: $(grep -o '"p50_suggest_ms": [0-9.]*\|"stage_ms": {[^}]*}' $O/bench_${TAG}_$v.err | tr '\n' ' ')"
        grep -i "k_sample\|k_tables" $O/stage_${TAG}_$v.txt | head -4
      done ;;
    rehearse)
      # the N > 1 flow with 2 ranks on the box's one GPU (gloo: RCCL takes one rank per device)
      for c in ${REH_CONFIGS:-3 4 5}; do
        step 600 $O/rehearse${c}_${TAG}.err env TPE_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + c)) bench.py --gpus 2 --config $c \
            --steps ${CFG_STEPS:-5} --warmup 2 --no-cpu-baseline --no-quantized --no-appending
        grep '^{' $O/rehearse${c}_${TAG}.err > $O/rehearse${c}_${TAG}.json; cat $O/rehearse${c}_${TAG}.json
      done ;;
    app5)
      # config 5 appending: cProfile of its steps, then the bench line
      step 300 $O/cfg5_app_prof_${TAG}.txt python tools/cfg5_app_prof.py ${STEPS:-8}
      head -30 $O/cfg5_app_prof_${TAG}.txt
      step 600 $O/cfg5app_${TAG}.err python bench.py --config 5 --appending --steps ${CFG_STEPS:-20} --warmup 2
      grep '^{' $O/cfg5app_${TAG}.err > $O/cfg5app_${TAG}.json; cat $O/cfg5app_${TAG}.json ;;
    trace5)
      # kernel trace of config 5 (APP5=--appending: the FMinIter flow)
      rm -rf $O/trace5_${TAG}
      step 600 $O/trace5_${TAG}.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace5_${TAG} -o run -- \
          python3 bench.py --config 5 ${APP5:-} --steps ${CFG_STEPS:-10} --warmup 2
      python3 tools/trace_summary.py $(find $O/trace5_${TAG} -name "*kernel_trace.csv") > $O/trace5_${TAG}_summary.txt
      head -30 $O/trace5_${TAG}_summary.txt ;;
    packtime)
      # the headline level's packer sections on the box's host CPU (no GPU; the
      # TPE_PACK_TRACE library from tools/build_pack_trace.sh; PACK_TOOL /
      # PACK_ARGS: another level, e.g. pack_time5.py "1000 100000 30" for config 5)
      for t in ${PACK_THREADS:-16}; do
        TPE_HOST_THREADS=$t TPE_PACK_LIB=$PWD/hyperopt_amd/libtpe_host_ptrace.so step 120 $O/packtime_${TAG}_$t.txt \
            python tools/${PACK_TOOL:-pack_time3.py} ${PACK_ARGS:-400}
        python3 tools/pack_sections.py $O/packtime_${TAG}_$t.txt | tee -a $O/packtime_${TAG}_$t.txt
      done ;;
    cfgprof)
      step 600 $O/cfgprof${CONFIG:-5}_${TAG}.txt python tools/config_prof.py ${CONFIG:-5} --steps ${STEPS:-5}
      head -45 $O/cfgprof${CONFIG:-5}_${TAG}.txt ;;
    hostprof)
      step 300 $O/hostprof_${TAG}.txt python tools/host_prof.py ${STEPS:-300}
      head -60 $O/hostprof_${TAG}.txt ;;
    phases)
      # host phases of one suggest per workload, under the kernel trace (device times)
      for w in ${PHASE_WL:-svm rf cfg2 app}; do
        rm -rf $O/phases_${TAG}_$w
        step 300 $O/phases_${TAG}_$w.txt rocprofv3 --kernel-trace --stats --output-format csv \
            -d $O/phases_${TAG}_$w -o run -- python3 tools/phase_prof.py $w ${STEPS:-200}
        python3 tools/trace_summary.py $(find $O/phases_${TAG}_$w -name "*kernel_trace.csv") >> $O/phases_${TAG}_$w.txt
        grep -v "^\[" $O/phases_${TAG}_$w.txt | head -20
      done ;;
    nativesplit)
      step 300 $O/nativesplit_${TAG}.txt python tools/native_split.py ${STEPS:-200} ${NS_ARGS:-}
      cat $O/nativesplit_${TAG}.txt ;;
    hostsplit)
      step 300 $O/hostsplit_${TAG}.txt python tools/host_split.py ${STEPS:-200}
      cat $O/hostsplit_${TAG}.txt ;;
    libab)
      for v in ${LIBS:-default}; do
        if [ "$v" = default ]; then lib=$PWD/hyperopt_amd/libtpe_hip.so; else lib=$PWD/hyperopt_amd/libtpe_hip_$v.so; fi
        step 300 $O/stage_${TAG}_$v.txt env TPE_HIP_LIB=$lib python tools/stage_bench.py ${REP:-20}
        step 300 $O/bench_${TAG}_$v.err env TPE_HIP_LIB=$lib python bench.py --no-cpu-baseline --no-quantized --no-config4 --steps ${AB_STEPS:-200}
        echo "$v: $(grep -o '"p50_suggest_ms": [0-9.]*\|"stage_ms": {[^}]*}' $O/bench_${TAG}_$v.err | tr '\n' ' ')"
        step 120 $O/phab_${TAG}_$v.txt env TPE_HIP_LIB=$lib python tools/phase_prof.py svm 300
        grep "p50\|phases" $O/phab_${TAG}_$v.txt
      done ;;
    pmcloop)
      # counters of the suggest flow itself (cold kernels between host phases)
      mkdir -p $O/pmcloop_${TAG}
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
                 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" \
                 "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
        nm=$(echo $grp | cut -d' ' -f1)
        rm -rf $O/pmcloop_${TAG}/$nm
        step 300 $O/pmcloop_${TAG}/$nm.log rocprofv3 --pmc $grp --kernel-trace --output-format csv \
            -d $O/pmcloop_${TAG}/$nm -o run -- python3 tools/suggest_loop.py 30
      done
      python3 tools/pmc_summary.py $O/pmcloop_${TAG} > $O/pmcloop_${TAG}/summary.json
      python3 -c "import json; d=json.load(open('$O/pmcloop_${TAG}/summary.json')); [print(k, json.dumps(v)) for k, v in d.items() if k.startswith('k_')]" ;;
    apitrace)
      rm -rf $O/api_${TAG}
      step 300 $O/api_${TAG}.log rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv \
          -d $O/api_${TAG} -o run -- python3 tools/suggest_loop.py 30
      python3 tools/api_timeline.py $O/api_${TAG} 2 > $O/api_${TAG}_timeline.txt
      cat $O/api_${TAG}_timeline.txt | head -120 ;;
    counters)
      step 120 $O/counters.txt rocprofv3 -L
      grep -o "SQ_[A-Z0-9_]*\|TCC_[A-Z0-9_]*\|TCP_[A-Z0-9_]*" $O/counters.txt | sort -u | tr '\n' ' ' | head -c 6000; echo ;;
    *)
      echo "unknown task $task"; exit 2 ;;
  esac
done
