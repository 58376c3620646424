#!/bin/bash
# host-only library with the packer's section clock (TPE_PACK_TRACE) for
# tools/pack_time4.py: TPE_PACK_LIB=hyperopt_amd/libtpe_host_ptrace.so
set -e
cd "$(dirname "$0")/.."
g++ -O3 -march=${TPE_HOST_MARCH:-x86-64-v2} -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -fno-trapping-math -DTPE_PACK_TRACE -I include hyperopt_amd/csrc/tpe_host.cpp hyperopt_amd/csrc/tpe_pool.cpp \
  -pthread -o hyperopt_amd/libtpe_host_ptrace.so
