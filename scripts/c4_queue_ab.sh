#!/bin/bash
# Config 4: queued (persistent) multi-wave grid vs one workgroup per item.
set -o pipefail
mkdir -p gpurun_out
for n in 256 512; do
  DEPPY_DEBUG_GRID=1 timeout -k 10 240 python -u scripts/config4.py $n 2 > gpurun_out/c4q_$n.json 2> gpurun_out/c4q_$n.err || exit 1
  DEPPY_NO_QUEUE=1 timeout -k 10 240 python -u scripts/config4.py $n 2 > gpurun_out/c4nq_$n.json 2> gpurun_out/c4nq_$n.err || exit 1
done
head -3 gpurun_out/c4q_256.err gpurun_out/c4q_512.err
for f in gpurun_out/c4q_256.json gpurun_out/c4nq_256.json gpurun_out/c4q_512.json gpurun_out/c4nq_512.json; do cut -c1-160 $f; done
