#!/bin/bash
# Device lowering: a measurement variant library (DEPPY_VARIANT_LIB=$2)
# against the product, config 2 call times (scripts/dl_probe.py), after the
# variant passes the device-lowering parity tests.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
DEPPY_VARIANT_LIB=$2 timeout -k 10 300 python -u -m pytest tests/test_device_lowering.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/var_tests.log 2>&1
rc=$?; tail -1 $OUT/var_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u scripts/dl_probe.py 2 10000 20 | sed 's/^/product /' || exit 1
  DEPPY_VARIANT_LIB=$2 timeout -k 10 200 python -u scripts/dl_probe.py 2 10000 20 | sed 's/^/variant /' || exit 1
done
