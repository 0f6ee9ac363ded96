#!/bin/bash
# Host-to-host pipeline sweep (config 2): zero-copy input, jobs in flight, chunk size.
out=gpurun_out/h2h_sweep.jsonl; : > $out
for zc in 1 0; do for depth in 2 3; do for chunk in 4096 2500; do
  DEPPY_ZC_IN=$zc DEPPY_CHUNK_PROBLEMS=$chunk timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu \
    --kernel-steps 0 --depth $depth > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print(json.dumps({'zc_in':$zc,'depth':$depth,'chunk':$chunk,'value':d['value'],'host':d['host_ms_per_step'],'kms':d['roofline']['kernel_ms_per_chunk'],'h2d':d['pcie']['h2d_GBs']}))" | tee -a $out
done; done; done
