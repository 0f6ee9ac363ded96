#!/bin/bash
# Round 3: fine LDS buckets (one per residency) vs the round-2 coarse ones.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03_gputest_d.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r03_gputest_d.log; [ $rc -eq 0 ] || exit 1
for cfg in 2 3 5; do
  for mode in fine coarse; do
    if [ $mode = coarse ]; then export DEPPY_CEILINGS=coarse DEPPY_BUCKET_MERGE=0.5; else unset DEPPY_CEILINGS DEPPY_BUCKET_MERGE; fi
    timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --kernel-steps 40 --no-cpu --e2e-steps 0 > gpurun_out/r03_bk_c${cfg}_$mode.json 2>&1 || exit 1
  done
done
unset DEPPY_CEILINGS DEPPY_BUCKET_MERGE
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_b4.json 2>gpurun_out/r03_b4.err
