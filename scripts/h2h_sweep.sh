#!/bin/bash
# Host-to-host pipeline sweep: chunk bytes per config (direct copies of
# page-locked 16-bit records where possible).
out=gpurun_out/h2h_sweep_r02c.jsonl; : > $out
for cfg in 5 4 2 3; do for cb in 64 128 256; do
  steps=20; [ $cfg = 3 ] && steps=12; [ $cfg = 5 ] && steps=8; [ $cfg = 4 ] && steps=4
  DEPPY_CHUNK_BYTES=$((cb<<20)) timeout -k 10 200 python bench.py --config $cfg \
    --steps $steps --warmup 8 --no-cpu --kernel-steps 0 > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print(json.dumps({'config':$cfg,'chunk_mb':$cb,'value':d['value'],'chunks':d['pipeline']['chunks_per_step'],'direct':d['direct_chunks_per_step'],'kms':d['pipeline']['kernel_ms_per_chunk'],'host':d['host_ms_per_step'],'h2d':d['pcie']['h2d_GBs']}))" | tee -a $out
done; done
