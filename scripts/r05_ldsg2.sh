#!/bin/bash
# Round 5: M_LDSG with 4 vs 8 wavefronts -- config 5's largest catalogs one at
# a time (ldsg_latency.py) and config 5 host to host / kernel only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
timeout -k 10 300 python scripts/ldsg_latency.py 20 300 > gpurun_out/r05/ldsg_lat_w4.txt 2>&1 || exit 1
DEPPY_VARIANT_LIB=libdeppy_hip_w8.so timeout -k 10 300 python scripts/ldsg_latency.py 20 300 > gpurun_out/r05/ldsg_lat_w8.txt 2>&1 || exit 1
cat gpurun_out/r05/ldsg_lat_w4.txt gpurun_out/r05/ldsg_lat_w8.txt
bash scripts/ab_env.sh 5 1 - DEPPY_VARIANT_LIB=libdeppy_hip_w8.so DEPPY_LDSG=0
