#!/bin/bash
# Round 3: GPU tests with the default library (2WL + row slots), config 4/5
# A/B over the multi-wave variants, driver-command bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03_gputest_c.log 2>&1
rc=$?; echo "default tests rc=$rc"; tail -2 gpurun_out/r03_gputest_c.log
[ $rc -eq 0 ] || exit 1
DEPPY_VARIANT_LIB=libdeppy_hip_slot.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "olm or multiwave or round_table or boundary or plain_int32 or wide" > gpurun_out/r03_gputest_slot.log 2>&1
echo "slot tests rc=$?"; tail -1 gpurun_out/r03_gputest_slot.log
for v in occ 2wl slot default; do
  lib=libdeppy_hip_$v.so; [ $v = default ] && lib=libdeppy_hip.so
  DEPPY_VARIANT_LIB=$lib timeout -k 10 150 python bench.py --config 4 --steps 4 --warmup 1 --no-cpu --e2e-steps 0 --kernel-steps 4 > gpurun_out/r03_c4_$v.json 2>&1 || exit 1
  DEPPY_VARIANT_LIB=$lib timeout -k 10 150 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu --e2e-steps 0 --kernel-steps 10 > gpurun_out/r03_c5_$v.json 2>&1 || exit 1
done
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_b3.json 2>gpurun_out/r03_b3.err || exit 1
timeout -k 10 120 python bench.py --config 6 --steps 20 --warmup 5 --no-cpu > gpurun_out/r03_b6b.json 2>&1
