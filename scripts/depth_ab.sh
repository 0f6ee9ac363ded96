#!/bin/bash
# Host-to-host jobs in flight (bench.py --depth) per config, 8 lanes per device.
set -o pipefail
mkdir -p gpurun_out/depth
for c in 2 3 5 4; do
  st=40; [ $c = 3 ] && st=16; [ $c = 5 ] && st=10; [ $c = 4 ] && st=6
  for d in 4 8; do
    timeout -k 10 300 python -u bench.py --config $c --steps $st --depth $d --kernel-steps 16 --no-cpu > gpurun_out/depth/c$c.d$d.json 2> gpurun_out/depth/c$c.d$d.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/depth/c$c.d$d.json')); print($c, $d, d['value'], d['kernel_only']['res_per_s'], d['deterministic'])"
  done
done
