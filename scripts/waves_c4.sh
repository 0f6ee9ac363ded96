#!/bin/bash
# Config 4: multi-wave group width A/B (DP_BIG_WAVES variants built with
# --tag): 256-catalog batch and single-catalog latency, parity vs the oracle.
set -o pipefail
mkdir -p gpurun_out
for v in "" _w1 _w2; do
  export DEPPY_VARIANT_LIB=libdeppy_hip$v.so
  timeout -k 10 240 python -u scripts/config4.py 256 3 > gpurun_out/c4$v.json 2> gpurun_out/c4$v.err || exit 1
  timeout -k 10 120 python -u scripts/config4.py 1 5 > gpurun_out/c4$v.lat.json 2>> gpurun_out/c4$v.err || exit 1
  echo "variant '$v' done"
done
