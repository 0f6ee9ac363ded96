#!/bin/bash
# Pipelined throughput vs workgroups per CU (LDS request padded): 0 = as built (9/CU for config 2),
# 19 KB -> 8/CU, 21 KB -> 7/CU, 24 KB -> 6/CU
mkdir -p gpurun_out/slots
for p in 0 19 21 24; do
  DEPPY_LDS_PAD_KB=$p timeout -k 10 60 python -u bench.py --no-cpu --steps 40 --warmup 8 > gpurun_out/slots/p$p.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/slots/p$p.log $p
done
