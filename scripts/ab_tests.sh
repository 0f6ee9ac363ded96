#!/bin/bash
# GPU parity tests per library variant, then the same-box A/B bench.
#   usage (via gpurun): bash scripts/ab_tests.sh <tag> "<configs>" <steps> lib1 lib2 ...
TAG=$1; CONFIGS=$2; STEPS=$3; shift 3
mkdir -p gpurun_out/$TAG
for lib in "$@"; do
  DEPPY_VARIANT_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.$lib.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/$TAG/tests.$lib.log)"
done
bash scripts/ab.sh $TAG "$CONFIGS" $STEPS "$@"
