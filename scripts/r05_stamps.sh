#!/bin/bash
# Round 5: phase stamps of the current build (diagnostic library
# libdeppy_hip_stamps.so: python -m deppy_amd.build --stamps): config 4 one
# catalog alone and 16 together, config 2 packed 10k; then the config-2 bench
# line (the pipelined SolveBatch path in solve_batch_api).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_stamps
mkdir -p $OUT


timeout -k 10 400 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 3 > $OUT/bench_c2.json 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); print('config 2', d['value'], d['kernel_only']['res_per_s'], d['end_to_end']['res_per_s'], d['solve_batch_api']['res_per_s'], d['host_lowering_res_per_s'])"
timeout -k 10 300 python -u scripts/pipe_timing.py 2 10000 > $OUT/pipe_timing.txt 2>&1 || exit 1; cat $OUT/pipe_timing.txt
