#!/bin/bash
# Host-to-host pipeline sweep: chunk size (problems and bytes) x jobs in flight,
# per config (direct copies of page-locked 16-bit records).
out=gpurun_out/h2h_sweep_r02b.jsonl; : > $out
for cfg in 2 3 5; do for chunk in 4096 16384 65536; do for cb in 24 64; do for depth in 3; do
  steps=30; [ $cfg = 3 ] && steps=12
  DEPPY_CHUNK_PROBLEMS=$chunk DEPPY_CHUNK_BYTES=$((cb<<20)) timeout -k 10 150 python bench.py --config $cfg \
    --steps $steps --warmup 4 --no-cpu --kernel-steps 0 --depth $depth > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print(json.dumps({'config':$cfg,'chunk':$chunk,'chunk_mb':$cb,'depth':$depth,'value':d['value'],'chunks':d['pipeline']['chunks_per_step'],'kms':d['pipeline']['kernel_ms_per_chunk'],'host':d['host_ms_per_step'],'h2d':d['pcie']['h2d_GBs']}))" | tee -a $out
done; done; done; done
