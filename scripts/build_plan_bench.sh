#!/bin/bash
# Builds scripts/plan_bench against the library's objects (after deppy_amd/build.py).
set -e
cd "$(dirname "$0")/.."
O=deppy_amd/_obj
/opt/rocm/bin/hipcc -O3 -std=c++17 -Iinclude -Ideppy_amd/csrc -x hip --offload-arch=gfx950 -c scripts/plan_bench.cpp -o /tmp/plan_bench.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/plan_bench.o $O/lower.cpp.o $O/gen.cpp.o $O/solve_launch.cpp.o \
  $O/solve_lds.hip.o $O/solve_lds_dense.hip.o $O/solve_split.hip.o $O/solve_split4.hip.o $O/solve_hbm.hip.o \
  -lpthread -o scripts/plan_bench
