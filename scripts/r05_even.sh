#!/bin/bash
# Round 5: the frontier dealt evenly over wavefronts (build) against the
# build before the barrier changes (libdeppy_hip_prev.so): GPU tests, config-4
# catalogs one at a time interleaved twice, configs 4 and 5 host to host, and
# where the SolveBatch path's time goes (scripts/pipe_timing.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_even
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/head_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/head_$rep.jsonl
  DEPPY_VARIANT_LIB=libdeppy_hip_prev.so timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/prev_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/prev_$rep.jsonl
done
for cfg in 4 5; do bash scripts/ab_env.sh $cfg 1 - DEPPY_VARIANT_LIB=libdeppy_hip_prev.so || exit 1; done
timeout -k 10 300 python -u scripts/pipe_timing.py 2 10000 > $OUT/pipe_timing.txt 2>&1 || exit 1; cat $OUT/pipe_timing.txt
