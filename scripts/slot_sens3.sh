#!/bin/bash
# config 3: throughput vs workgroups per CU (LDS padded: 0 = natural, 10 KB -> 16/CU, 16 KB -> 10/CU, 20 KB -> 8/CU)
mkdir -p gpurun_out/slots3
for p in 0 10 16 20; do
  DEPPY_LDS_PAD_KB=$p timeout -k 10 120 python -u bench.py --no-cpu --config 3 --steps 20 --warmup 8 > gpurun_out/slots3/p$p.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/slots3/p$p.log $p
done
