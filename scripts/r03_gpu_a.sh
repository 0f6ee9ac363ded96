#!/bin/bash
# Round 3: GPU tests (default library), 2WL variant parity on the multi-wave
# tests, driver-command benches, config 4 A/B (occurrence lists vs 2WL).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03_gputest.log 2>&1
echo "default tests rc=$?"; tail -2 gpurun_out/r03_gputest.log
DEPPY_VARIANT_LIB=libdeppy_hip_2wl.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "olm or multiwave or round_table or boundary or config5 or plain_int32 or wide or generated" > gpurun_out/r03_gputest_2wl.log 2>&1
echo "2wl tests rc=$?"; tail -2 gpurun_out/r03_gputest_2wl.log
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_b1.json 2>gpurun_out/r03_b1.err || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/r03_b2.json 2>&1 || exit 1
timeout -k 10 150 python bench.py --config 4 --steps 4 --warmup 1 --no-cpu --e2e-steps 0 --kernel-steps 4 > gpurun_out/r03_c4_occ.json 2>&1 || exit 1
DEPPY_VARIANT_LIB=libdeppy_hip_2wl.so timeout -k 10 150 python bench.py --config 4 --steps 4 --warmup 1 --no-cpu --e2e-steps 0 --kernel-steps 4 > gpurun_out/r03_c4_2wl.json 2>&1 || exit 1
timeout -k 10 120 python bench.py --config 6 --steps 20 --warmup 5 > gpurun_out/r03_b6.json 2>&1
