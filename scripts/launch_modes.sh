#!/bin/bash
# Throughput of the pipelined bench under launch-placement variants (diagnostic env knobs).
mkdir -p gpurun_out/lm
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 60 python -u bench.py --no-cpu --steps 40 --warmup 4 --depth $D > gpurun_out/lm/$tag.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['serial_ms_per_step'])" gpurun_out/lm/$tag.log $tag
}
for D in 3 4 8; do
  run split_d$D DEPPY_BUCKET_MERGE=0
  run merge_d$D DEPPY_BUCKET_MERGE=0.5
  run serial_d$D DEPPY_LANE_SERIAL=1
done
