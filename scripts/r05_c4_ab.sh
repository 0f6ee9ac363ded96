#!/bin/bash
# Round 5, config 4: 2-byte device-built watch entries (layout.hpp went_bytes)
# against the 8-byte {row, row_info} entries (variant libdeppy_hip_went8.so,
# -DDP_WENT=8).  GPU tests of the build, then the same 20 catalogs one at a
# time (scripts/c4_latency.py) interleaved twice, then config 4 and 5 host to
# host / kernel only.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_c4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/head_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/head_$rep.jsonl
  DEPPY_VARIANT_LIB=libdeppy_hip_went8.so timeout -k 10 300 python -u scripts/c4_latency.py 20 > $OUT/went8_$rep.jsonl 2>&1 || exit 1
  tail -1 $OUT/went8_$rep.jsonl
done
bash scripts/ab_env.sh 4 1 - DEPPY_VARIANT_LIB=libdeppy_hip_went8.so || exit 1
bash scripts/ab_env.sh 5 1 - DEPPY_VARIANT_LIB=libdeppy_hip_went8.so || exit 1
