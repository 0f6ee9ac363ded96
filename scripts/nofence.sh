#!/bin/bash
mkdir -p gpurun_out/nf
export DEPPY_VARIANT_LIB=libdeppy_hip_nofence.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nf/t.log 2>&1; tail -1 gpurun_out/nf/t.log
timeout -k 10 120 python -u bench.py --steps 40 --warmup 8 --cpu-seconds 1 > gpurun_out/nf/b.log 2>&1 || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('nofence', d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['verified_bit_exact_vs_oracle'])" gpurun_out/nf/b.log
unset DEPPY_VARIANT_LIB
timeout -k 10 120 python -u bench.py --steps 40 --warmup 8 --cpu-seconds 1 > gpurun_out/nf/b0.log 2>&1 || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('fence', d['value'], d['ms_per_step'], d['serial_ms_per_step'], d['verified_bit_exact_vs_oracle'])" gpurun_out/nf/b0.log
