#!/usr/bin/env bash
# PMC counter passes on the bench workload (one rocprofv3 run per counter group).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  rm -rf gpurun_out/pmc/$name
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/$name.out 2> gpurun_out/pmc/$name.err
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU &&
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json &&
python3 -c "import json; print(json.dumps(json.load(open('gpurun_out/pmc/summary.json'))['traffic'], indent=1))"
