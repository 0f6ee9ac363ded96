#!/bin/bash
# Round 5: GPU tests (pipelined SolveBatch path included); config-4 catalogs
# one at a time on 8-wave (default) and 4-wave groups (DEPPY_C4_FLAGS=4,
# DP_OPT_FORCE_MID); config 2 bench line (solve_batch_api: the pipelined
# SolveBatch path).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_misc
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/c4_latency.py 10 > $OUT/c4_w8.jsonl 2>&1 || exit 1
tail -1 $OUT/c4_w8.jsonl
DEPPY_C4_FLAGS=4 timeout -k 10 300 python -u scripts/c4_latency.py 10 > $OUT/c4_w4.jsonl 2>&1 || exit 1
tail -1 $OUT/c4_w4.jsonl
timeout -k 10 400 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/bench_c2.json 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); print('config 2', d['value'], d['kernel_only']['res_per_s'], d['end_to_end'], d['solve_batch_api'], d['host_lowering_res_per_s'])"
