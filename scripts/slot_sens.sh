#!/bin/bash
# Pipelined throughput vs workgroups per CU (LDS request padded: 22 KB -> 7/CU, 23 -> 6, 27 -> 5, 32 -> 5, 40 -> 4)
mkdir -p gpurun_out/slots
for p in 0 23 27 40; do
  DEPPY_LDS_PAD_KB=$p timeout -k 10 60 python -u bench.py --no-cpu --steps 40 --warmup 8 > gpurun_out/slots/p$p.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/slots/p$p.log $p
done
