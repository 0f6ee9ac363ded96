#!/bin/bash
# Records' H2D on copy streams (default) vs on the compute streams, per config.
set -o pipefail
mkdir -p gpurun_out/cs
for c in 5 2 4; do
  st=40; [ $c = 5 ] && st=10; [ $c = 4 ] && st=6
  for v in 1 0; do
    DEPPY_COPY_STREAM=$v timeout -k 10 300 python -u bench.py --config $c --steps $st --kernel-steps 8 --no-cpu > gpurun_out/cs/c$c.$v.json 2> gpurun_out/cs/c$c.$v.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/cs/c$c.$v.json')); print($c, 'copy_stream=$v', d['value'], d['kernel_only']['res_per_s'], d['pcie']['h2d_GBs'], d['deterministic'])"
  done
done
