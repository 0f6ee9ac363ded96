#!/bin/bash
# LDS-path variants: natural occupancy (and bit-exact check)
mkdir -p gpurun_out/impv
for lib in libdeppy_hip.so libdeppy_hip_imp32.so libdeppy_hip_i32w128.so; do
  DEPPY_VARIANT_LIB=$lib timeout -k 10 120 python -u bench.py --steps 40 --warmup 8 --cpu-seconds 1 > gpurun_out/impv/$lib.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['verified_bit_exact_vs_oracle'])" gpurun_out/impv/$lib.log "$lib"
done
