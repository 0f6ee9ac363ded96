#!/bin/bash
mkdir -p gpurun_out/mw
for lib in libdeppy_hip.so libdeppy_hip_mw6.so libdeppy_hip_mw8.so; do
  for c in 3 2; do
    DEPPY_VARIANT_LIB=$lib timeout -k 10 150 python -u bench.py --config $c --steps 20 --warmup 8 --cpu-seconds 1 > gpurun_out/mw/$lib.$c.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['verified_bit_exact_vs_oracle'])" gpurun_out/mw/$lib.$c.log "$lib config$c"
  done
done
