#!/bin/bash
# Throughput vs the LDS percentile the bulk launch is sized to (DEPPY_LDS_PCT)
mkdir -p gpurun_out/pct
for p in 0 99 95 90; do
  DEPPY_LDS_PCT=$p timeout -k 10 60 python -u bench.py --no-cpu --steps 40 --warmup 8 > gpurun_out/pct/p$p.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['serial_ms_per_step'])" gpurun_out/pct/p$p.log $p
done
