#!/bin/bash
# Config-4 time and parity: release library (8-wave groups) vs a 16-wave variant
mkdir -p gpurun_out/c4v
for lib in libdeppy_hip.so libdeppy_hip_w16.so; do
  DEPPY_VARIANT_LIB=$lib timeout -k 10 150 python -u scripts/config4.py 256 3 > gpurun_out/c4v/$lib.log 2>&1 || exit 1
  echo $lib $(tail -1 gpurun_out/c4v/$lib.log | cut -c1-230)
done
