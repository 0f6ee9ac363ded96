#!/bin/bash
# Round 5: multi-wave kernels capped at two waves per SIMD, against the build
# before the round's barrier changes (libdeppy_hip_prev.so): GPU tests, configs
# 5 and 4 host to host / kernel only, config-4 catalogs one at a time.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05_cap
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for cfg in 5 4; do bash scripts/ab_env.sh $cfg 2 - DEPPY_VARIANT_LIB=libdeppy_hip_prev.so || exit 1; done
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/head_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/head_$rep.jsonl
  DEPPY_VARIANT_LIB=libdeppy_hip_prev.so timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/prev_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/prev_$rep.jsonl
done
