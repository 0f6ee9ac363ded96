#!/bin/bash
# forced multi-wave parity in the diagnostic builds (race study)
mkdir -p gpurun_out/race2
for lib in libdeppy_hip_stamps.so libdeppy_hip_stamps_w16.so; do
  for cfg in "2 60 1" "2 60 2" "5 60 1" "3 300 1"; do
    tag=$(echo $lib.$cfg | tr ' ' _)
    DEPPY_STAMPS=1 DEPPY_STAMPS_LIB=$lib timeout -k 10 90 python -u scripts/check_probe.py $cfg > gpurun_out/race2/$tag.log 2>&1 || exit 1
    echo $tag $(tail -1 gpurun_out/race2/$tag.log | cut -c1-60)
  done
done
