#!/bin/bash
# Round 3: GPU tests (latency path, occurrence-list default), driver bench,
# configs 3-6 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03_gputest_e.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r03_gputest_e.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_b5.json 2>gpurun_out/r03_b5.err || exit 1
DEPPY_FAST_PATH=0 timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > gpurun_out/r03_b5_nofast.json 2>&1 || exit 1
for cfg in 3 4 5 6; do
  timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --kernel-steps 20 --cpu-seconds 5 > gpurun_out/r03_c${cfg}.json 2>&1 || exit 1
done
